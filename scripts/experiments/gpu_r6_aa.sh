#!/bin/bash
# Round 6: k_emb_final as an adjacency launch + a parameter launch for packed grids (the parameter
# workgroups at 152 instead of 190 VGPRs: 3 waves per SIMD instead of 2) -- packed fits at R = 16
# bitwise split vs one launch, and the R = 128 grid A/B (D4IC twice, TST once).
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_FITS_R=16 COMPARE_FITS_CFGS=d4ic,c1k4,c4
REDCLIFF_EMB_FINAL_SPLIT=0 step aa_dump_one 400 python scripts/compare_fits.py dump gpurun_out/aa_one.npz
REDCLIFF_EMB_FINAL_SPLIT=1 step aa_dump_split 400 python scripts/compare_fits.py dump gpurun_out/aa_split.npz
step aa_compare 120 python scripts/compare_fits.py compare gpurun_out/aa_one.npz gpurun_out/aa_split.npz
rm -f gpurun_out/aa_one.npz gpurun_out/aa_split.npz
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2; do
  REDCLIFF_EMB_FINAL_SPLIT=0 step aa_grid_one_$i 300 python bench.py $GR
  REDCLIFF_EMB_FINAL_SPLIT=1 step aa_grid_split_$i 300 python bench.py $GR
done
REDCLIFF_EMB_FINAL_SPLIT=0 step aa_grid_one_c4 300 python bench.py $GR --config c4
REDCLIFF_EMB_FINAL_SPLIT=1 step aa_grid_split_c4 300 python bench.py $GR --config c4
