#!/bin/bash
# Round 3 start: the round-2 HEAD on a fresh box (the driver's r02 GPU run was skipped).
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step a_tests 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread --durations=25
step a_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step a_bench 400 python -u bench.py --steps 20 --warmup 5
kill $HB
