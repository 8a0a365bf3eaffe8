#!/bin/bash
# Round 4: factor leads' adjacency-L1 loops and the embedder node blocks' LDS loops unrolled (LDS reads in flight):
# vector path, single-fit A/B interleaved, phase trace
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4az
step az_dump4 300 python -u scripts/compare_fits.py dump gpurun_out/r4az/fcur4.npz
for i in 1 2 3; do
step az_single_cur$i 200 python -u scripts/ab_single.py --tag cur
step az_single_prev$i 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev0.so python -u scripts/ab_single.py --tag prev
done
step az_trace 200 python -u scripts/phase_trace.py --config d4ic
step az_tests 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_forked.py tests/test_gpu_fit_golden.py tests/test_gpu_data_parallel.py
kill $HB
