#!/bin/bash
# Round 4: fit-level parity (envelopes incl. the published-lr D4IC fit) and the packed-fit host split
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step l_fit 700 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_fit_golden.py
step l_pf_split 400 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --host-split --cprofile
kill $HB
