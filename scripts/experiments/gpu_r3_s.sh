#!/bin/bash
# Round 3: HBM counter passes (FETCH_SIZE / WRITE_SIZE, separate runs) of the single-fit bench leg
# and of the R = 128 grid step on the current build (bench.py's roofline.traffic reads them), the
# default bench line and its kernel stats.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
S="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-north-star --no-kernel-times --replicas 1 --fit-replicas 0 --dp-leg-batch 0"
G="python scripts/grid_step.py --replicas 128 --steps 3"
F="--kernel-include-regex k_ --output-format csv"
step s_fetch 150 rocprofv3 --pmc FETCH_SIZE $F -d gpurun_out/pmc_s_fetch -o run -- $S
step s_write 150 rocprofv3 --pmc WRITE_SIZE $F -d gpurun_out/pmc_s_write -o run -- $S
step g_fetch 150 rocprofv3 --pmc FETCH_SIZE $F -d gpurun_out/pmc_g_fetch -o run -- $G
step g_write 150 rocprofv3 --pmc WRITE_SIZE $F -d gpurun_out/pmc_g_write -o run -- $G
step s_bench 400 python bench.py
step s_stats 400 rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d gpurun_out/stats_s -o run -- python bench.py --no-cpu-baseline --steps 100 --warmup 10
kill $HB
