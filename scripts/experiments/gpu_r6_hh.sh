#!/bin/bash
# Round 6: k_emb_final's batched parameter path requesting the parameters and moments together
# with the gradients (RC_EF_PMV_FIRST=1, lib_pmvfirst) against after them (the tree) -- packed fits
# bitwise (R = 16 and 8), R = 128 grid A/B; kernel-trace summaries of the tree's R = 128 grids.
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_FITS_CFGS=d4ic,c1k4,c4
for R in 16 8; do
  COMPARE_FITS_R=$R step hh_dump_0_$R 300 python scripts/compare_fits.py dump gpurun_out/hh_0.npz
  COMPARE_FITS_R=$R REDCLIFF_HIP_LIB=scripts/bin/lib_pmvfirst.so step hh_dump_1_$R 300 python scripts/compare_fits.py dump gpurun_out/hh_1.npz
  step hh_compare_$R 120 python scripts/compare_fits.py compare gpurun_out/hh_0.npz gpurun_out/hh_1.npz
  rm -f gpurun_out/hh_0.npz gpurun_out/hh_1.npz
done
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2; do
  for cfg in c4 d4ic; do
    step hh_grid_0_${cfg}_$i 300 python bench.py $GR --config $cfg
    REDCLIFF_HIP_LIB=scripts/bin/lib_pmvfirst.so step hh_grid_1_${cfg}_$i 300 python bench.py $GR --config $cfg
  done
done
for cfg in d4ic c4; do
  REDCLIFF_FORK=0 step hh_stats_$cfg 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hh/$cfg -o run -- python scripts/grid_step.py --replicas 128 --steps 20 --config $cfg
  REDCLIFF_FORK=0 REDCLIFF_HIP_LIB=scripts/bin/lib_pmvfirst.so step hh_stats1_$cfg 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hh1/$cfg -o run -- python scripts/grid_step.py --replicas 128 --steps 20 --config $cfg
done
rm -f gpurun_out/hh/*/run_kernel_trace.csv gpurun_out/hh1/*/run_kernel_trace.csv
