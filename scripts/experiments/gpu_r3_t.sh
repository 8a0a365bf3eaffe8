#!/bin/bash
# Round 3: the TST-shaped single-fit step (configs[3]'s per-rank work): bench line, kernel stats,
# phase timeline; the DP step breakdown at global batch 128.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
C="python bench.py --config c4 --steps 200 --warmup 20 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0"
step t_bench 300 $C
step t_stats 300 rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d gpurun_out/stats_t -o run -- $C
step t_trace 200 python -u scripts/phase_trace.py --config c4
step t_dp 300 python -u scripts/dp_profile.py --batch 128
kill $HB
