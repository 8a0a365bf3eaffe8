#!/bin/bash
# Round 4: packed fit host trims (precomputed module list, batched restore): tests + host split
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step n_tests 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pack_fit.py tests/test_gpu_fit_modes.py tests/test_gpu_checkpoint.py
step n_pf_split 400 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --host-split
step n_pf_split2 400 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --host-split --cprofile
kill $HB
