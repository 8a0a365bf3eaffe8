#!/bin/bash
# Round 5 final-tree evidence (final: after the data-parallel register fix, r5ao): the driver's bench command; the single-fit (D4IC) bench leg under
# rocprofv3 --kernel-trace --stats and its FETCH / WRITE passes (the line's roofline kernel); the
# R = 128 grid (one stream) kernel stats and passes; GPU suite + smoke
source "$(dirname "$0")/../gpu_steps.sh"
step v_bench 600 python bench.py
S="python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0"
step v_stats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v/stats -o run -- $S
step v_fetch 240 timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/v/fetch -o run -- $S
step v_write 240 timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/v/write -o run -- $S
G="python scripts/grid_step.py --replicas 128 --steps 20"
REDCLIFF_FORK=0 step v_gstats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v/gstats -o run -- $G
REDCLIFF_FORK=0 step v_gfetch 240 timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/v/gfetch -o run -- $G
REDCLIFF_FORK=0 step v_gwrite 240 timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/v/gwrite -o run -- $G
rm -f gpurun_out/v/*/run_kernel_trace.csv
step v_suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA --durations=10
step v_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
