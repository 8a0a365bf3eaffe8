#!/bin/bash
# Round 3, end: full GPU suite and the driver's default bench line on the final tree
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step f4_suite 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --durations=5
step f4_bench 500 python bench.py
kill $HB
