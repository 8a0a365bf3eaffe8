#!/bin/bash
# Round 5: k_fac_bwd_s16 at 4 waves per SIMD (scripts/bin/lib_s16w4.so, 232 bytes of scratch) against the
# 3-wave default: R = 128 grid kernel times (one stream) and bitwise packed fits
source "$(dirname "$0")/../gpu_steps.sh"
S="python scripts/grid_sweep.py --replicas 128 --steps 30 --rounds 2 --kernel-times --settings [{\"REDCLIFF_FORK\":\"0\"}]"
for rep in 1 2; do
  step w_cur_$rep 300 $S
  REDCLIFF_HIP_LIB=scripts/bin/lib_s16w4.so step w_w4_$rep 300 $S
done
COMPARE_FITS_R=32 step w_dump_cur 300 python scripts/compare_fits.py dump gpurun_out/wcur.npz
COMPARE_FITS_R=32 REDCLIFF_HIP_LIB=scripts/bin/lib_s16w4.so step w_dump_w4 300 python scripts/compare_fits.py dump gpurun_out/ww4.npz
step w_cmp 60 python scripts/compare_fits.py compare gpurun_out/wcur.npz gpurun_out/ww4.npz
rm -f gpurun_out/wcur.npz gpurun_out/ww4.npz
