#!/bin/bash
# Round 3: the driver's default bench line and its kernel statistics on the current build
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step f1_bench 600 python bench.py
step f1_stats 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f1_stats -o run -- python bench.py --no-cpu-baseline --steps 100 --warmup 10
kill $HB
