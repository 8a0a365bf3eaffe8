#!/bin/bash
# Round 5: node staging issues all factor-side dL/dw partial rounds together (p <= 16, K > 4):
# bitwise whole packed fits (previous build vs current; c4 has K = 9) and the TST step timeline
source "$(dirname "$0")/../gpu_steps.sh"
P=scripts/bin/lib_prev_r5c.so
for R in 1 4; do
  COMPARE_FITS_CFGS=c4,c1k4 COMPARE_FITS_R=$R REDCLIFF_HIP_LIB=$P step ac_dump_prev_$R 300 python scripts/compare_fits.py dump gpurun_out/fprev_$R.npz
  COMPARE_FITS_CFGS=c4,c1k4 COMPARE_FITS_R=$R step ac_dump_cur_$R 300 python scripts/compare_fits.py dump gpurun_out/fcur_$R.npz
  step ac_cmp_$R 60 python scripts/compare_fits.py compare gpurun_out/fprev_$R.npz gpurun_out/fcur_$R.npz
done
rm -f gpurun_out/fprev_*.npz gpurun_out/fcur_*.npz
K="--steps 50 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times --config c4 --preheat-s 0"
step ac_kt 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ac/kt -o run -- python bench.py $K
f=$(ls gpurun_out/ac/kt/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && step ac_timeline 60 python scripts/step_timeline.py "$f" --steps 3
rm -rf gpurun_out/ac/kt
step ac_tests 600 python -u -m pytest tests/test_gpu_forked.py tests/test_gpu_fit_golden.py tests/test_gpu_replicas.py -v --timeout 300 --timeout-method thread -rA
