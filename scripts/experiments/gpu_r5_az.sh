#!/bin/bash
# k_lemb_prep_win with T_0 stored in runs of F floats: R = 128 grid kernel stats and write pass,
# the driver's bench command, GPU suite, smoke.
source "$(dirname "$0")/../gpu_steps.sh"
G="python scripts/grid_step.py --replicas 128 --steps 20"
REDCLIFF_FORK=0 step az_gstats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/az/gstats -o run -- $G
REDCLIFF_FORK=0 step az_gwrite 240 timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/az/gwrite -o run -- $G
rm -f gpurun_out/az/*/run_kernel_trace.csv
step az_suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA --durations=10
step az_bench 600 python bench.py
step az_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
