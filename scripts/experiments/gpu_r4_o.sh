#!/bin/bash
# Round 4: evaluation-side kernels (gc_norms staged, gc_dots per sample, cos values 4 windows per
# workgroup) and the packed-fit host trims: bitwise fit records vs the HEAD build, tests, profile
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4o
step o_dump_prev 300 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python -u scripts/compare_fits.py dump gpurun_out/r4o/fprev.npz
step o_dump_cur 300 python -u scripts/compare_fits.py dump gpurun_out/r4o/fcur.npz
step o_compare 120 python -u scripts/compare_fits.py compare gpurun_out/r4o/fprev.npz gpurun_out/r4o/fcur.npz
step o_tests 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pack_fit.py tests/test_gpu_fit_modes.py tests/test_gpu_checkpoint.py tests/test_gpu_parity.py tests/test_gpu_fit_golden.py
step o_pf_split 400 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --host-split
step o_pf_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4o/prof -o pf -- python3 scripts/pack_fit_profile.py --replicas 128 --epochs 40
kill $HB
