#!/bin/bash
# Round 6: k_fac_mix in 128-thread workgroups (REDCLIFF_MIX_NT) --
# plus k_fac_bwd_s16 timing-only variants (RC_S16_EXP 1 / 2 / 3: no Adam arithmetic / no matrix-core passes /
# neither); whole packed fits bitwise against the previous build (compare_fits, R = 8: the
# matrix-core factor chain, D4IC / C1(K=4) / TST), the R = 128 grid A/B, and the pack trace's phase marks.
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_FITS_R=8 COMPARE_FITS_CFGS=d4ic,c1k4,c4
REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so step l_dump_prev 300 python scripts/compare_fits.py dump gpurun_out/l_prev.npz
step l_dump_cur 300 python scripts/compare_fits.py dump gpurun_out/l_cur.npz
step l_compare 120 python scripts/compare_fits.py compare gpurun_out/l_prev.npz gpurun_out/l_cur.npz
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2; do
  REDCLIFF_MIX_NT=256 step l_grid_nt256_$i 300 python bench.py $GR
  step l_grid_nt128_$i 300 python bench.py $GR
done
for v in 1 2 3; do
  REDCLIFF_HIP_LIB=scripts/bin/lib_s16exp$v.so step l_grid_s16exp$v 300 python bench.py $GR
done
REDCLIFF_FORK=0 step l_trace 300 python scripts/phase_trace_pack.py --replicas 128 --steps 6
rm -f gpurun_out/l_prev.npz gpurun_out/l_cur.npz
step l_fit_lag64 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fit_golden.py -k lag64 -s
