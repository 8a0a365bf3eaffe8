#!/bin/bash
# Round 6 tree: kernel stats (single fit, R = 128 grid with the factor chain on one stream, C5) and the HBM
# counter passes (FETCH_SIZE / WRITE_SIZE in separate runs) of the single fit and the grid.
source "$(dirname "$0")/../gpu_steps.sh"
S="python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --c5-steps 0"
G="python scripts/grid_step.py --replicas 128 --steps 20"
C5="python bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --c5-steps 0 --no-kernel-times"
step f_stats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f/stats -o run -- $S
REDCLIFF_FORK=0 step f_gstats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f/gstats -o run -- $G
step f_c5stats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f/c5stats -o run -- $C5
step f_fetch 240 timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/f/fetch -o run -- $S
step f_write 240 timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/f/write -o run -- $S
REDCLIFF_FORK=0 step f_gfetch 240 timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/f/gfetch -o run -- $G
REDCLIFF_FORK=0 step f_gwrite 240 timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/f/gwrite -o run -- $G
rm -f gpurun_out/f/*/run_kernel_trace.csv
