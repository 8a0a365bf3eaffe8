#!/bin/bash
# Round 4: software-pipelined recompute in k_fac_bwd_s16: bitwise packed fits at R=8 (matrix-core
# factor path) vs the HEAD build, grid step A/B interleaved, kernel stats
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4ab
step ab_dump_prev 300 env COMPARE_FITS_R=8 REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python -u scripts/compare_fits.py dump gpurun_out/r4ab/fprev8.npz
step ab_dump_cur 300 env COMPARE_FITS_R=8 python -u scripts/compare_fits.py dump gpurun_out/r4ab/fcur8.npz
step ab_compare 120 python -u scripts/compare_fits.py compare gpurun_out/r4ab/fprev8.npz gpurun_out/r4ab/fcur8.npz
for i in 1 2; do
step ab_grid_cur$i 200 python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2 --settings '[{}]'
step ab_grid_prev$i 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2 --settings '[{}]'
done
step ab_prof_cur 200 env REDCLIFF_FORK=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ab/cur -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step ab_prof_prev 200 env REDCLIFF_FORK=0 REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ab/prev -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
kill $HB
