#!/bin/bash
# Round 5 final-tree evidence (after the latency work, r5ac-r5ak): the driver's bench command; the single-fit (D4IC) bench leg under
# rocprofv3 --kernel-trace --stats and its FETCH / WRITE passes (the line's roofline kernel); the
# R = 128 grid (one stream) kernel stats and passes; GPU suite + smoke
source "$(dirname "$0")/../gpu_steps.sh"
step u_bench 600 python bench.py
S="python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0"
step u_stats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/u/stats -o run -- $S
step u_fetch 240 timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/u/fetch -o run -- $S
step u_write 240 timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/u/write -o run -- $S
G="python scripts/grid_step.py --replicas 128 --steps 20"
REDCLIFF_FORK=0 step u_gstats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/u/gstats -o run -- $G
REDCLIFF_FORK=0 step u_gfetch 240 timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/u/gfetch -o run -- $G
REDCLIFF_FORK=0 step u_gwrite 240 timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/u/gwrite -o run -- $G
rm -f gpurun_out/u/*/run_kernel_trace.csv
step u_suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA --durations=10
step u_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
