#!/bin/bash
# Round 5: GEMM core K step (RC_GEMM_K 16 -> 32 / 64: fewer dependent operand round trips per tile)
# on the R = 128 grid (its six embedder GEMMs ~27 us each), kernel stats, bitwise whole packed fits
source "$(dirname "$0")/../gpu_steps.sh"
S="python scripts/grid_sweep.py --replicas 128 --steps 30 --rounds 2 --kernel-times --settings [{\"REDCLIFF_FORK\":\"0\"}]"
for rep in 1 2; do
  step q_cur_$rep 300 $S
  REDCLIFF_HIP_LIB=scripts/bin/lib_gk32.so step q_gk32_$rep 300 $S
  REDCLIFF_HIP_LIB=scripts/bin/lib_gk64.so step q_gk64_$rep 300 $S
done
P="timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv"
step q_stats_cur 200 $P -d gpurun_out/q/cur -o run -- python scripts/grid_step.py --replicas 128 --steps 20
for v in gk32 gk64; do
  REDCLIFF_HIP_LIB=scripts/bin/lib_$v.so step q_stats_$v 200 $P -d gpurun_out/q/$v -o run -- python scripts/grid_step.py --replicas 128 --steps 20
done
rm -f gpurun_out/q/*/run_kernel_trace.csv
COMPARE_FITS_R=32 step q_dump_cur 300 python scripts/compare_fits.py dump gpurun_out/qcur.npz
COMPARE_FITS_R=32 REDCLIFF_HIP_LIB=scripts/bin/lib_gk64.so step q_dump_gk64 300 python scripts/compare_fits.py dump gpurun_out/qgk64.npz
step q_cmp 60 python scripts/compare_fits.py compare gpurun_out/qcur.npz gpurun_out/qgk64.npz
rm -f gpurun_out/qcur.npz gpurun_out/qgk64.npz
REDCLIFF_HIP_LIB=scripts/bin/lib_gk64.so step q_tests 300 python -u -m pytest tests/test_gpu_generic.py -k gemm -v --timeout 300 --timeout-method thread -rA
