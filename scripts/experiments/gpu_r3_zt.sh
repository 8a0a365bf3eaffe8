#!/bin/bash
# Round 3: where a packed grid-search fit's wall clock goes (R = 128, 40 epochs, the bench's
# fits/hour unit), with a host cProfile of one unwrapped fit
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step zt_packfit 500 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --train-batches 8 --cprofile
kill $HB
