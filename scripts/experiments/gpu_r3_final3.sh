#!/bin/bash
# Round 3 (final build, after the merged-lead split and the matrix-core factor backward): the
# driver's default bench line, its kernel stats, HBM counter passes of the single fit; TST with
# the split-lead step forced on / off
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
S="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-north-star --no-kernel-times --replicas 1 --fit-replicas 0 --dp-leg-batch 0"
F="--kernel-include-regex k_ --output-format csv"
step f3_fetch 150 rocprofv3 --pmc FETCH_SIZE $F -d gpurun_out/f3_pmc_s_fetch -o run -- $S
step f3_write 150 rocprofv3 --pmc WRITE_SIZE $F -d gpurun_out/f3_pmc_s_write -o run -- $S
step f3_bench 500 python bench.py
step f3_stats 400 rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d gpurun_out/f3_stats -o run -- python bench.py --no-cpu-baseline --steps 100 --warmup 10
B="python bench.py --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0"
step f3_c4_split0 200 env REDCLIFF_SPLIT_LEAD=0 $B --config c4
step f3_c4_split1 200 env REDCLIFF_SPLIT_LEAD=1 $B --config c4
step f3_dpbench 300 python bench.py --mode dp --dp-batch 128 --steps 300 --warmup 30
kill $HB
