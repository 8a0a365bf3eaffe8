#!/bin/bash
# Round 4: wave-per-window cos values, wave-per-sample GC dots, pipelined GC norms: bitwise fit
# records vs the HEAD build, tests (incl. the whole-state envelope criterion), packed-fit profile
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4p
step p_dump_cur 300 python -u scripts/compare_fits.py dump gpurun_out/r4p/fcur.npz
step p_compare 120 python -u scripts/compare_fits.py compare gpurun_out/r4o/fprev.npz gpurun_out/r4p/fcur.npz
step p_tests 900 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_fit_golden.py tests/test_gpu_pack_fit.py tests/test_gpu_parity.py
step p_pf_split 400 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --host-split
step p_pf_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4p/prof -o pf -- python3 scripts/pack_fit_profile.py --replicas 128 --epochs 40
kill $HB
