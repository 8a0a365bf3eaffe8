#!/bin/bash
# Round 3: packed fit with the module modes written directly vs torch's recursive .eval()
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step zu_torch_eval 400 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --train-batches 8 --torch-eval
step zu_direct 400 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --train-batches 8
step zu_torch_eval2 400 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --train-batches 8 --torch-eval
step zu_direct2 400 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --train-batches 8
step zu_tests 400 python -u -m pytest tests/test_gpu_pack_fit.py tests/test_gpu_fit_modes.py -v --timeout 120 --timeout-method thread
kill $HB
