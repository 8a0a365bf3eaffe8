#!/bin/bash
# Round 6 round-end evidence on the final tree: the driver's sequence (GPU suite, smoke, default bench
# line), kernel-trace summaries (single fit, R = 128 grid with the factor chain on one stream, C5), and
# the HBM counter passes (FETCH_SIZE / WRITE_SIZE in separate runs) of the single fit and the grid.
source "$(dirname "$0")/../gpu_steps.sh"
step z_suite 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA --durations=15
step z_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step z_bench 600 python bench.py
S="python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --c5-steps 0"
G="python scripts/grid_step.py --replicas 128 --steps 20"
C5="python bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --c5-steps 0 --no-kernel-times"
step z_stats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/z/stats -o run -- $S
REDCLIFF_FORK=0 step z_gstats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/z/gstats -o run -- $G
step z_c5stats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/z/c5stats -o run -- $C5
step z_fetch 240 timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/z/fetch -o run -- $S
step z_write 240 timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/z/write -o run -- $S
REDCLIFF_FORK=0 step z_gfetch 240 timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/z/gfetch -o run -- $G
REDCLIFF_FORK=0 step z_gwrite 240 timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/z/gwrite -o run -- $G
rm -f gpurun_out/z/*/run_kernel_trace.csv
