#!/bin/bash
# Round 4: side-stream GC tracking vs one stream, interleaved on one box
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
for i in 1 2 3; do
step af_side$i 300 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40
step af_one$i 300 env REDCLIFF_PACK_SIDE=0 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40
done
kill $HB
