#!/bin/bash
# Round 2: the whole GPU suite on the final build, then smoke().
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step r2_suite2 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step r2_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
kill $HB
