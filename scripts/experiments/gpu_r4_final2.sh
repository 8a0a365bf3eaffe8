#!/bin/bash
# Round 4, final tree (after the multi-rank coordination and packed-fit changes): full GPU suite,
# smoke, the driver's default bench line twice
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step f2_suite 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread --durations=5
step f2_smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step f2_bench 600 python bench.py --steps 20 --warmup 5
step f2_bench2 600 python bench.py --steps 20 --warmup 5
kill $HB
