#!/bin/bash
# Round 6: k_lemb_head with 4 / 2 windows per wave (the default for packs of >= 8 replicas) against
# one (REDCLIFF_HEAD_WPW=1) -- packed fits bitwise (R = 16: GEMM embedder), R = 128 grid A/B.
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_FITS_R=16 COMPARE_FITS_CFGS=d4ic,c1k4,c4
step gg_dump_4 300 python scripts/compare_fits.py dump gpurun_out/gg_4.npz
REDCLIFF_HEAD_WPW=1 step gg_dump_1 300 python scripts/compare_fits.py dump gpurun_out/gg_1.npz
step gg_compare 120 python scripts/compare_fits.py compare gpurun_out/gg_4.npz gpurun_out/gg_1.npz
rm -f gpurun_out/gg_4.npz gpurun_out/gg_1.npz
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2; do
  for cfg in c4 d4ic; do
    for w in 1 2 4; do
      REDCLIFF_HEAD_WPW=$w step gg_grid_${w}_${cfg}_$i 300 python bench.py $GR --config $cfg
    done
  done
done
step gg_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gg_prof -o run -- python bench.py $GR --config d4ic
