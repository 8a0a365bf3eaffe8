#!/bin/bash
# Round 5 final tree (wave GEMM core for every product): C5 single fit (GEMM embedder) A/B against the
# LDS-tiled core, the driver's bench command, single-fit and R = 128 grid kernel stats and HBM passes,
# GPU suite, smoke.
source "$(dirname "$0")/../gpu_steps.sh"
C5="python bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0"
REDCLIFF_GEMM_CORE=mfma step ax_c5_mfma 240 $C5
step ax_c5_def 240 $C5
step ax_bench 600 python bench.py
S="python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0"
step ax_stats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ax/stats -o run -- $S
G="python scripts/grid_step.py --replicas 128 --steps 20"
REDCLIFF_FORK=0 step ax_gstats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ax/gstats -o run -- $G
REDCLIFF_FORK=0 step ax_gfetch 240 timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ax/gfetch -o run -- $G
REDCLIFF_FORK=0 step ax_gwrite 240 timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/ax/gwrite -o run -- $G
rm -f gpurun_out/ax/*/run_kernel_trace.csv
step ax_suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA --durations=10
step ax_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
