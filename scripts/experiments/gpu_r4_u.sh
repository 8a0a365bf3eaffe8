#!/bin/bash
# Round 4: forked packed steps from 32 replicas, k_emb_final 8 elements per thread from 96:
# bitwise fit records, replica / pack / fork tests, grid step, packed-fit profile
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4u
step u_dump_cur 300 python -u scripts/compare_fits.py dump gpurun_out/r4u/fcur.npz
step u_tests 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py tests/test_gpu_forked.py
step u_grid 200 python -u scripts/grid_step.py --replicas 128 --steps 40
step u_pf_split 400 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --host-split
kill $HB
