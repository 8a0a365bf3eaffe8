#!/bin/bash
# GEMM tile choice: GPU suite, then C5 with auto tiles vs forced 64x64
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --config c5 --no-cpu-baseline --steps 50 --warmup 5 --replicas 1 > gpurun_out/c5_auto.log 2>&1 || exit 1
REDCLIFF_GEMM_TILE=64 timeout -k 10 200 python -u bench.py --config c5 --no-cpu-baseline --steps 50 --warmup 5 --replicas 1 > gpurun_out/c5_t64.log 2>&1 || exit 1
REDCLIFF_GEMM_TILE=32 timeout -k 10 200 python -u bench.py --config c5 --no-cpu-baseline --steps 50 --warmup 5 --replicas 1 > gpurun_out/c5_t32.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_c5 -o run -- python bench.py --config c5 --no-cpu-baseline --no-kernel-times --steps 30 --warmup 5 --replicas 1 > gpurun_out/kt_c5.log 2>&1
