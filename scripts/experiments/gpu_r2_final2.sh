#!/bin/bash
# Round 2 close: the whole GPU suite, smoke(), the driver's bench command and its kernel-trace
# stats on the final build.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step f2_tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step f2_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step f2_bench 500 python -u bench.py --steps 20 --warmup 5
step f2_kstats 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kstats_f2 -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
kill $HB
