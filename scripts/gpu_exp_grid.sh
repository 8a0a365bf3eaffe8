#!/bin/bash
# GPU suite twice (replica packs on one stream), then the D4IC bench (+grid) and C1(K=4)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 200 python -u -m pytest tests/test_gpu_replicas.py -q --timeout 150 --timeout-method thread > gpurun_out/rep2.log 2>&1
timeout -k 10 200 python -u -m pytest tests/test_gpu_replicas.py -q --timeout 150 --timeout-method thread > gpurun_out/rep3.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_d4ic.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --config c5 --no-cpu-baseline --steps 50 --warmup 5 --replicas 1 > gpurun_out/bench_c5.log 2>&1 || exit 1
exit 0
