#!/bin/bash
# Round 2 end: the whole GPU suite, the driver's bench command, and the kernel-trace stats of
# the same command on the final build.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step r2_end_tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step r2_end_bench 500 python -u bench.py --steps 20 --warmup 5
step r2_end_kstats 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kstats_end -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
kill $HB
