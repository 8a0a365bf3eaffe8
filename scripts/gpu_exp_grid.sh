#!/bin/bash
# packed-grid forward tuning: windows per forward workgroup (default 8 at R >= 8) vs 4; GPU suite
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline --steps 300 --warmup 30 --replicas 32 --grid-steps 100"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 $B > gpurun_out/grid_sbdef.log 2>&1 || exit 1
REDCLIFF_EMB_SB=4 timeout -k 10 200 $B > gpurun_out/grid_sb4.log 2>&1 || exit 1
REDCLIFF_EMB_SB=16 timeout -k 10 200 $B > gpurun_out/grid_sb16.log 2>&1 || exit 1
