#!/bin/bash
# Iteration pass: all GPU parity tests, the C5 stress bench and the phase traces.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 200 --warmup 20 --replicas 1 > gpurun_out/bench_d4ic.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config c5 --no-cpu-baseline --steps 50 --warmup 5 --replicas 1 > gpurun_out/bench_c5.log 2>&1 && \
timeout -k 10 120 python -u scripts/phase_trace.py --config d4ic > gpurun_out/trace_d4ic.log 2>&1 && \
timeout -k 10 120 python -u scripts/phase_trace.py --config c5 > gpurun_out/trace_c5.log 2>&1
