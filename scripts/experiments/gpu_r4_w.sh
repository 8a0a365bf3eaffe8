#!/bin/bash
# Round 4, checkpoint: full GPU suite, smoke, and the driver's default bench line on the current tree
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step w_suite 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread --durations=5
step w_smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step w_bench 500 python bench.py --steps 20 --warmup 5
kill $HB
