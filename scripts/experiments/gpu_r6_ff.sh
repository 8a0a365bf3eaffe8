#!/bin/bash
# Round 6: k_fac_mix requesting A's column and b1's Adam state at its start (RC_MIX_EARLY=1,
# lib_mixearly) against where they are used (the tree) -- packed fits bitwise (R = 8), R = 128 grid
# A/B at TST and D4IC.
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_FITS_R=8 COMPARE_FITS_CFGS=d4ic,c1k4,c4
step ff_dump_0 300 python scripts/compare_fits.py dump gpurun_out/ff_0.npz
REDCLIFF_HIP_LIB=scripts/bin/lib_mixearly.so step ff_dump_1 300 python scripts/compare_fits.py dump gpurun_out/ff_1.npz
step ff_compare 120 python scripts/compare_fits.py compare gpurun_out/ff_0.npz gpurun_out/ff_1.npz
rm -f gpurun_out/ff_0.npz gpurun_out/ff_1.npz
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2; do
  for cfg in c4 d4ic; do
    step ff_grid_0_${cfg}_$i 300 python bench.py $GR --config $cfg
    REDCLIFF_HIP_LIB=scripts/bin/lib_mixearly.so step ff_grid_1_${cfg}_$i 300 python bench.py $GR --config $cfg
  done
done
