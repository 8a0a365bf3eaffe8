#!/bin/bash
# Round 3: embedder-backward sub-block products on the matrix cores, short-contraction kernels v4 --
# full GPU suite, single-fit phase timeline, default bench line and its kernel stats.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step q_suite 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --durations=10
step q_trace 200 python -u scripts/phase_trace.py --config d4ic
step q_bench 400 python bench.py --no-cpu-baseline
step q_stats 400 rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d gpurun_out/stats_q -o run -- python bench.py --no-cpu-baseline --steps 100 --warmup 10
kill $HB
