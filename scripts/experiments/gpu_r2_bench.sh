#!/bin/bash
# the driver's bench command on the current build
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step r2_bench 500 python -u bench.py --steps 20 --warmup 5
kill $HB
