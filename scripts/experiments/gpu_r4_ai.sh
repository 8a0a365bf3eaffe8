#!/bin/bash
# Round 4: short-contraction factor backward with the epilogue in the accumulator layout
# (k_fac_bwd_s16e, 4 waves per SIMD): bitwise packed fits at R=8 against the previous build's
# dump, grid step A/B interleaved, kernel stats, factor-path tests
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4ai
step ai_dump8 300 env COMPARE_FITS_R=8 python -u scripts/compare_fits.py dump gpurun_out/r4ai/fcur8.npz
for i in 1 2; do
step ai_grid_cur$i 200 python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2 --settings '[{}]'
step ai_grid_prev$i 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2 --settings '[{}]'
done
step ai_prof_cur 200 env REDCLIFF_FORK=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ai/cur -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step ai_prof_prev 200 env REDCLIFF_FORK=0 REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ai/prev -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step ai_tests 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py tests/test_gpu_forked.py tests/test_gpu_parity.py tests/test_gpu_data_parallel.py
kill $HB
