#!/bin/bash
# Round 5 final tree (single-replica products back on the LDS-tiled GEMM core): C5 default against
# the forced wave core, the grid step's kernel stats, GPU suite, smoke.
source "$(dirname "$0")/../gpu_steps.sh"
C5="python bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0"
step ay_c5_def 240 $C5
REDCLIFF_GEMM_CORE=wave step ay_c5_wave 240 $C5
G="python scripts/grid_step.py --replicas 128 --steps 20"
REDCLIFF_FORK=0 step ay_gstats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ay/gstats -o run -- $G
rm -f gpurun_out/ay/*/run_kernel_trace.csv
step ay_suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA --durations=10
step ay_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
