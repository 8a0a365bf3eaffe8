#!/bin/bash
# Round 6: k_fac_fwd_s16 requesting its operands two blocks ahead (RC_FWD_AHEAD=2, lib_ahead2) against
# one (the tree) -- packed fits bitwise, R = 128 grid A/B alternated three times (D4IC) and once (TST).
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_FITS_R=8 COMPARE_FITS_CFGS=d4ic,c4
step t_dump_1 300 python scripts/compare_fits.py dump gpurun_out/t_1.npz
REDCLIFF_HIP_LIB=scripts/bin/lib_ahead2.so step t_dump_2 300 python scripts/compare_fits.py dump gpurun_out/t_2.npz
step t_compare 120 python scripts/compare_fits.py compare gpurun_out/t_1.npz gpurun_out/t_2.npz
rm -f gpurun_out/t_1.npz gpurun_out/t_2.npz
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2 3; do
  step t_grid_a1_$i 300 python bench.py $GR
  REDCLIFF_HIP_LIB=scripts/bin/lib_ahead2.so step t_grid_a2_$i 300 python bench.py $GR
done
step t_grid_a1_c4 300 python bench.py $GR --config c4
REDCLIFF_HIP_LIB=scripts/bin/lib_ahead2.so step t_grid_a2_c4 300 python bench.py $GR --config c4
