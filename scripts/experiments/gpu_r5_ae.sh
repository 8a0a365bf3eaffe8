#!/bin/bash
# Round 5: one staging round where the common shapes took two or three (forward: S, W_i, fc2 with
# more loads per thread; node staging: fc2 at K M1 = 576), same bits.  Bitwise whole packed fits
# against the previous build, single-fit steps previous vs current, phase traces, kernel tests.
source "$(dirname "$0")/../gpu_steps.sh"
P=scripts/bin/lib_prev_r5e.so
for R in 1; do
  COMPARE_FITS_CFGS=c4,c1k4,d4ic,c5 COMPARE_FITS_R=$R REDCLIFF_HIP_LIB=$P step ae_dump_prev_$R 300 python scripts/compare_fits.py dump gpurun_out/fprev_$R.npz
  COMPARE_FITS_CFGS=c4,c1k4,d4ic,c5 COMPARE_FITS_R=$R step ae_dump_cur_$R 300 python scripts/compare_fits.py dump gpurun_out/fcur_$R.npz
  step ae_cmp_$R 60 python scripts/compare_fits.py compare gpurun_out/fprev_$R.npz gpurun_out/fcur_$R.npz
done
rm -f gpurun_out/fprev_*.npz gpurun_out/fcur_*.npz
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
for cfg in c1k4 c4 d4ic; do
  REDCLIFF_HIP_LIB=$P step ae_prev_${cfg}_$rep 200 $B --config $cfg
  step ae_cur_${cfg}_$rep 200 $B --config $cfg
done
done
step ae_trace_c1k4 200 python scripts/phase_trace.py --config c1k4
step ae_trace_c4 200 python scripts/phase_trace.py --config c4
step ae_tests 600 python -u -m pytest tests/test_gpu_forked.py tests/test_gpu_fit_golden.py tests/test_gpu_replicas.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -rA
