#!/bin/bash
# Round 6: k_fac_mix staging 2 (the tree) / 4 / 8 predictions per thread per round of loads --
# packed fits bitwise (R = 8) and the R = 128 grid A/B at TST and D4IC.
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_FITS_R=8 COMPARE_FITS_CFGS=d4ic,c4
step cc_dump_2 300 python scripts/compare_fits.py dump gpurun_out/cc_2.npz
REDCLIFF_HIP_LIB=scripts/bin/lib_mixu8.so step cc_dump_8 300 python scripts/compare_fits.py dump gpurun_out/cc_8.npz
step cc_compare 120 python scripts/compare_fits.py compare gpurun_out/cc_2.npz gpurun_out/cc_8.npz
rm -f gpurun_out/cc_2.npz gpurun_out/cc_8.npz
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for cfg in c4 d4ic; do
  step cc_grid_u2_$cfg 300 python bench.py $GR --config $cfg
  REDCLIFF_HIP_LIB=scripts/bin/lib_mixu4.so step cc_grid_u4_$cfg 300 python bench.py $GR --config $cfg
  REDCLIFF_HIP_LIB=scripts/bin/lib_mixu8.so step cc_grid_u8_$cfg 300 python bench.py $GR --config $cfg
done
