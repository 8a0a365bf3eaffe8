#!/bin/bash
# Round 6: k_fac_mix in 64-thread workgroups (REDCLIFF_MIX_NT=64; block sums over the 256-thread
# window layout) against 128 (the default) -- packed fits bitwise against the round's previous
# build for both, and the R = 128 grid A/B (D4IC three times, TST once).
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_FITS_R=8 COMPARE_FITS_CFGS=d4ic,c1k4,c4
REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so step u_dump_prev 300 python scripts/compare_fits.py dump gpurun_out/u_prev.npz
step u_dump_128 300 python scripts/compare_fits.py dump gpurun_out/u_128.npz
REDCLIFF_MIX_NT=64 step u_dump_64 300 python scripts/compare_fits.py dump gpurun_out/u_64.npz
step u_compare_128 120 python scripts/compare_fits.py compare gpurun_out/u_prev.npz gpurun_out/u_128.npz
step u_compare_64 120 python scripts/compare_fits.py compare gpurun_out/u_prev.npz gpurun_out/u_64.npz
rm -f gpurun_out/u_prev.npz gpurun_out/u_128.npz gpurun_out/u_64.npz
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2 3; do
  step u_grid_128_$i 300 python bench.py $GR
  REDCLIFF_MIX_NT=64 step u_grid_64_$i 300 python bench.py $GR
done
step u_grid_128_c4 300 python bench.py $GR --config c4
REDCLIFF_MIX_NT=64 step u_grid_64_c4 300 python bench.py $GR --config c4
