#!/bin/bash
# Round 4: k_emb_final batched parameter path with its one-record gradients requested together and
# the W_i slice sums 8 loads per round: bitwise packed fits, grid A/B interleaved, kernel stats
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4ax
step ax_dump8 300 env COMPARE_FITS_R=8 python -u scripts/compare_fits.py dump gpurun_out/r4ax/fcur8.npz
for i in 1 2; do
step ax_grid_cur$i 200 python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2 --settings '[{}]'
step ax_grid_prev$i 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2 --settings '[{}]'
done
step ax_prof_cur 200 env REDCLIFF_FORK=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ax/cur -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step ax_prof_prev 200 env REDCLIFF_FORK=0 REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ax/prev -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step ax_tests 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py tests/test_gpu_forked.py
kill $HB
