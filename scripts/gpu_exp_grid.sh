#!/bin/bash
# GPU suite + bench (single D4IC fit + packed grid) + C5 after the stream-policy change
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --config c5 --no-cpu-baseline --steps 50 --warmup 5 --replicas 1 > gpurun_out/bench_c5.log 2>&1 || exit 1
