#!/bin/bash
# Round 6: kernel-trace summary of the R = 128 TST-shaped grid step (the reference TST grid's class),
# factor chain on one stream.
source "$(dirname "$0")/../gpu_steps.sh"
G="python scripts/grid_step.py --replicas 128 --steps 20 --config c4"
REDCLIFF_FORK=0 step bb_tst_stats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bb/tst -o run -- $G
rm -f gpurun_out/bb/*/run_kernel_trace.csv
