#!/bin/bash
# Round 2: the packed grid at R = 128 on one stream (default) and forked (factor chain on a
# second stream, REDCLIFF_FORK=1), grid and fits/hour legs.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
G="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-north-star --no-kernel-times"
step gf_one 400 $G
REDCLIFF_FORK=1 step gf_fork 400 $G
kill $HB
