#!/bin/bash
# Round 5: RcDiv32 -- the host's division multipliers as 32-bit ceil(2^32 / d) (one v_mul_hi_u32, one
# scalar register each; the 64-bit ones added to the hot kernels' scalar-register spills).  Bitwise whole
# fits (R = 1 and 4), single-fit steps against the previous build, phase traces, the GPU suite.
source "$(dirname "$0")/../gpu_steps.sh"
P=scripts/bin/lib_prev_r5k.so
COMPARE_FITS_CFGS=c4,c1k4,d4ic,c5 COMPARE_FITS_R=1 REDCLIFF_HIP_LIB=$P step ak_dump_prev 300 python scripts/compare_fits.py dump gpurun_out/fprev_1.npz
COMPARE_FITS_CFGS=c4,c1k4,d4ic,c5 COMPARE_FITS_R=1 step ak_dump_cur 300 python scripts/compare_fits.py dump gpurun_out/fcur_1.npz
step ak_cmp 60 python scripts/compare_fits.py compare gpurun_out/fprev_1.npz gpurun_out/fcur_1.npz
rm -f gpurun_out/fprev_*.npz gpurun_out/fcur_*.npz
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
for cfg in c1k4 c4 d4ic; do
  REDCLIFF_HIP_LIB=$P step ak_prev_${cfg}_$rep 200 $B --config $cfg
  step ak_cur_${cfg}_$rep 200 $B --config $cfg
done
done
step ak_trace_c1k4 200 python scripts/phase_trace.py --config c1k4
step ak_trace_c4 200 python scripts/phase_trace.py --config c4
COMPARE_FITS_CFGS=c4,c1k4 COMPARE_FITS_R=4 REDCLIFF_HIP_LIB=$P step ak_dump_prev4 300 python scripts/compare_fits.py dump gpurun_out/fprev_4.npz
COMPARE_FITS_CFGS=c4,c1k4 COMPARE_FITS_R=4 step ak_dump_cur4 300 python scripts/compare_fits.py dump gpurun_out/fcur_4.npz
step ak_cmp4 60 python scripts/compare_fits.py compare gpurun_out/fprev_4.npz gpurun_out/fcur_4.npz
rm -f gpurun_out/fprev_*.npz gpurun_out/fcur_*.npz
step ak_suite 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x
