#!/bin/bash
# Round 4: kernel trace of an R=128 packed D4IC fit (epoch-level split of training vs evaluation)
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4ak
step ak_trace 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4ak/tr -o p -- python3 scripts/pack_fit_profile.py --replicas 128 --epochs 10
kill $HB
