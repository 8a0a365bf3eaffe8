#!/bin/bash
# Round 4: network-major y slots (ABI 8) -- full GPU suite, the driver's bench command twice,
# kernel stats of the same command
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4am
step am_tests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests
step am_bench_a 400 python -u bench.py --steps 20 --warmup 5
step am_bench_b 400 python -u bench.py --steps 20 --warmup 5
step am_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4am/prof -o b -- python3 bench.py --steps 20 --warmup 5
kill $HB
