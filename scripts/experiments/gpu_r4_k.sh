#!/bin/bash
# Round 4: packed-fit host split (enqueue / wait / digest per epoch) and host cProfile, R=128 D4IC
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step k_pf_split 400 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --host-split --cprofile
kill $HB
