#!/bin/bash
# Round 4: GC tracking on a side stream beside validation: bitwise fit records (R=4 and R=8),
# pack / fit-mode / checkpoint tests, packed-fit timing
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4ae
step ae_dump4 300 python -u scripts/compare_fits.py dump gpurun_out/r4ae/fcur4.npz
step ae_dump8 300 env COMPARE_FITS_R=8 python -u scripts/compare_fits.py dump gpurun_out/r4ae/fcur8.npz
step ae_tests 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pack_fit.py tests/test_gpu_fit_modes.py tests/test_gpu_checkpoint.py
step ae_pf1 300 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --host-split
step ae_pf2 300 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --host-split
kill $HB
