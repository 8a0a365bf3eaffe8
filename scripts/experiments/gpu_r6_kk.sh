#!/bin/bash
# Round 6: HBM traffic of the R = 128 TST grid's kernels (FETCH_SIZE / WRITE_SIZE, separate passes).
source "$(dirname "$0")/../gpu_steps.sh"
G="python scripts/grid_step.py --replicas 128 --steps 5 --config c4"
REDCLIFF_FORK=0 step kk_fetch 240 timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/kk/fetch -o run -- $G
REDCLIFF_FORK=0 step kk_write 240 timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/kk/write -o run -- $G
