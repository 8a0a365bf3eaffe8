#!/bin/bash
# Round 4: factor leads' channel loop (adjacency L1) and mixing loop unrolled:
# vector path, single-fit A/B interleaved, phase trace
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4bb
step bb_dump4 300 python -u scripts/compare_fits.py dump gpurun_out/r4bb/fcur4.npz
for i in 1 2 3; do
step bb_single_cur$i 200 python -u scripts/ab_single.py --tag cur
step bb_single_prev$i 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev2.so python -u scripts/ab_single.py --tag prev
done
step bb_trace 200 python -u scripts/phase_trace.py --config d4ic
step bb_tests 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_forked.py tests/test_gpu_fit_golden.py tests/test_gpu_data_parallel.py
kill $HB
