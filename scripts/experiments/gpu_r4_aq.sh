#!/bin/bash
# Round 4: packed-fit epoch composition on the current build (kernel trace + unprofiled host split)
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4aq
step aq_split 300 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --host-split
step aq_trace 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4aq/tr -o p -- python3 scripts/pack_fit_profile.py --replicas 128 --epochs 10
kill $HB
