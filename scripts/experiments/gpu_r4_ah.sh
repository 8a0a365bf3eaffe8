#!/bin/bash
# Round 4: k_emb_final's parameter workgroups in packs with every run's loads in one round:
# bitwise packed fits (R=8, R=4) vs earlier dumps, grid step A/B interleaved, kernel stats, tests
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4ah
step ah_dump8 300 env COMPARE_FITS_R=8 python -u scripts/compare_fits.py dump gpurun_out/r4ah/fcur8.npz
step ah_dump4 300 python -u scripts/compare_fits.py dump gpurun_out/r4ah/fcur4.npz
for i in 1 2; do
step ah_grid_cur$i 200 python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2 --settings '[{}]'
step ah_grid_prev$i 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2 --settings '[{}]'
done
step ah_prof_cur 200 env REDCLIFF_FORK=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ah/cur -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step ah_prof_prev 200 env REDCLIFF_FORK=0 REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ah/prev -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step ah_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py tests/test_gpu_forked.py
kill $HB
