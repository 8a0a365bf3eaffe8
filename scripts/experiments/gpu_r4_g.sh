#!/bin/bash
# Round 4: workgroup timelines (trace build) of the single-fit step at the north-star, TST and D4IC shapes
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step g_trace_c1k4 200 python scripts/phase_trace.py --config c1k4
step g_trace_c4 200 python scripts/phase_trace.py --config c4
step g_trace_d4ic 200 python scripts/phase_trace.py --config d4ic
step g_stats_c1k4 200 rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d gpurun_out/stats_g -o run -- python bench.py --config c1k4 --steps 100 --warmup 10 --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --no-cpu-baseline --no-north-star
kill $HB
