#!/bin/bash
# Round 4: XCD-aware order of the per-window embedder kernels (k_lemb_*, k_cos_values) in packs:
# bitwise packed fits, in-process grid A/B, kernel stats, packed-fit A/B
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4at
step at_dump8 300 env COMPARE_FITS_R=8 python -u scripts/compare_fits.py dump gpurun_out/r4at/fcur8.npz
step at_sweep 500 python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 4 --settings '[{}, {"REDCLIFF_EMB_XCD": "0"}]'
step at_prof_on 200 env REDCLIFF_FORK=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4at/son -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step at_prof_off 200 env REDCLIFF_FORK=0 REDCLIFF_EMB_XCD=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4at/soff -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
for i in 1 2; do
step at_pack_on$i 300 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40
step at_pack_off$i 300 env REDCLIFF_EMB_XCD=0 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40
done
step at_tests 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py tests/test_gpu_forked.py tests/test_gpu_generic.py
kill $HB
