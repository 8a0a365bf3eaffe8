#!/bin/bash
# Round 4: y slots network-major ([slot][network][window]): bitwise packed fits (R=8 matrix-core
# short kernels, R=4 vector path) against the previous build's dumps, grid and single-fit A/B
# interleaved, kernel stats, HBM write/fetch passes, full GPU suite
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4al
step al_dump8 300 env COMPARE_FITS_R=8 python -u scripts/compare_fits.py dump gpurun_out/r4al/fcur8.npz
step al_dump4 300 python -u scripts/compare_fits.py dump gpurun_out/r4al/fcur4.npz
for i in 1 2; do
step al_grid_cur$i 200 python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2 --settings '[{}]'
step al_grid_prev$i 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2 --settings '[{}]'
step al_single_cur$i 200 python -u scripts/ab_single.py --tag cur
step al_single_prev$i 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python -u scripts/ab_single.py --tag prev
done
step al_prof_cur 200 env REDCLIFF_FORK=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4al/cur -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step al_prof_prev 200 env REDCLIFF_FORK=0 REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4al/prev -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step al_pmc_write 120 timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r4al/pw -o w -- python3 scripts/grid_step.py --replicas 128 --steps 5
step al_pmc_fetch 120 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r4al/pf -o f -- python3 scripts/grid_step.py --replicas 128 --steps 5
step al_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests
kill $HB
