#!/bin/bash
# Kernel trace of the packed grid-search run (R = 32 replicas per launch).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_grid -o run -- python bench.py --no-cpu-baseline --no-kernel-times --steps 10 --warmup 2 --replicas 32 --grid-steps 50 > gpurun_out/kt_grid.log 2>&1
