#!/bin/bash
# Round 4: parameter-only speculative saves when no replica can stop: bitwise fit records (with
# early stops and rollbacks), pack-fit tests, packed-fit profile
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4aa
step aa_dump_cur 300 python -u scripts/compare_fits.py dump gpurun_out/r4aa/fcur.npz
step aa_tests 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pack_fit.py tests/test_gpu_fit_modes.py tests/test_gpu_checkpoint.py
step aa_pf1 300 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --host-split
step aa_pf2 300 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --host-split
kill $HB
