#!/bin/bash
# kernel traces (timelines) of the packed grid (R = 32, D4IC) and of the C5 single fit
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_grid -o run -- python bench.py --no-cpu-baseline --no-kernel-times --steps 10 --warmup 2 --replicas 32 --grid-steps 50 > gpurun_out/kt_grid.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_c5 -o run -- python bench.py --config c5 --no-cpu-baseline --no-kernel-times --steps 30 --warmup 5 --replicas 1 > gpurun_out/kt_c5.log 2>&1
