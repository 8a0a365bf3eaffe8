#!/bin/bash
# Round-end evidence: bench line (CPU baseline included), kernel-trace summaries of the single
# fit and of the packed grid, FETCH / WRITE counter passes of the single-fit bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B1="python bench.py --no-cpu-baseline --no-kernel-times --steps 50 --warmup 5 --replicas 1"
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o run -- python bench.py --no-cpu-baseline --steps 300 --warmup 30 --replicas 1 > gpurun_out/kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_grid -o run -- python bench.py --no-cpu-baseline --no-kernel-times --steps 10 --warmup 2 --replicas 32 --grid-steps 50 > gpurun_out/kt_grid.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- $B1 > gpurun_out/pmc1.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- $B1 > gpurun_out/pmc2.log 2>&1
