#!/bin/bash
# Round 6: k_fac_mix with its window weights / targets / group-norm partials / output-bias state requested
# in the staging round -- whole packed fits bitwise against the previous build (compare_fits, R = 8: the
# matrix-core factor chain, D4IC / C1(K=4) / TST), the R = 128 grid A/B, and the pack trace's phase marks.
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_FITS_R=8 COMPARE_FITS_CFGS=d4ic,c1k4,c4
REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so step k_dump_prev 300 python scripts/compare_fits.py dump gpurun_out/k_prev.npz
step k_dump_cur 300 python scripts/compare_fits.py dump gpurun_out/k_cur.npz
step k_compare 120 python scripts/compare_fits.py compare gpurun_out/k_prev.npz gpurun_out/k_cur.npz
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2; do
  REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so step k_grid_prev_$i 300 python bench.py $GR
  step k_grid_cur_$i 300 python bench.py $GR
done
REDCLIFF_FORK=0 step k_trace 300 python scripts/phase_trace_pack.py --replicas 128 --steps 6
rm -f gpurun_out/k_prev.npz gpurun_out/k_cur.npz
