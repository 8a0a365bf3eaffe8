#!/bin/bash
# Round 4, start: GPU suite on the build-id tree, steady-state timing study, driver-style bench line
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step a_suite 700 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --durations=10
step a_steady 200 python -u scripts/steady_state.py
step a_bench20 400 python bench.py --steps 20 --warmup 5
kill $HB
