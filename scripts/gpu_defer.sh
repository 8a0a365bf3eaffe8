#!/bin/bash
# combine-variant check: bitwise tests, then the D4IC bench with the separate combine launch
# (default) and with the in-place read by k_emb_final (REDCLIFF_DEFER=2)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_replicas.py -v --timeout 200 --timeout-method thread > gpurun_out/pytest_rep.log 2>&1 && \
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_d1.log 2>&1 && \
REDCLIFF_DEFER=2 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_d2.log 2>&1 && \
REDCLIFF_DEFER=2 timeout -k 10 200 python -u bench.py --config c1k4 --no-cpu-baseline --replicas 1 > gpurun_out/bench_c1_d2.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config c1k4 --no-cpu-baseline --replicas 1 > gpurun_out/bench_c1_d1.log 2>&1
