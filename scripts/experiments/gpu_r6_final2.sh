#!/bin/bash
# Round 6 final tree (after the k_emb_final split for wide packs): GPU suite, smoke, default bench
# line, and the kernel-trace summary of the R = 128 grid (factor chain on one stream) and of a TST pack.
source "$(dirname "$0")/../gpu_steps.sh"
step f2_suite 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA --durations=15
step f2_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step f2_bench 600 python bench.py
G="python scripts/grid_step.py --replicas 128 --steps 20"
REDCLIFF_FORK=0 step f2_gstats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f2/gstats -o run -- $G
rm -f gpurun_out/f2/*/run_kernel_trace.csv
