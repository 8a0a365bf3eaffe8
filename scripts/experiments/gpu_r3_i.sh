#!/bin/bash
# Round 3 (resumed session): full GPU suite, smoke, default bench line and its kernel stats on HEAD.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step i_suite 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --durations=15
step i_smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step i_bench 400 python bench.py
step i_stats 400 rocprofv3 --kernel-trace --stats --kernel-include-regex ^k_ --output-format csv -d gpurun_out/stats_i -o run -- python bench.py --no-cpu-baseline
kill $HB
