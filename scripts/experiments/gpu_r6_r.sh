#!/bin/bash
# Round 6: interleaved chains in the windowed embedder kernels (k_lemb_win_bwd's dx_bn rows, four at a
# time; k_lemb_prep_win's T_i items, RC_PREP_CHAINS at a time) -- whole packed fits at R = 16 (the
# GEMM-shaped embedder) bitwise against the round's previous build, then the R = 128 grid A/B
# (last commit / 4 / 2 / 1 prep chains) and the pack trace's phase marks.
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_FITS_R=16 COMPARE_FITS_CFGS=d4ic,c1k4,c4
REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so step r_dump_prev 400 python scripts/compare_fits.py dump gpurun_out/r_prev.npz
step r_dump_cur 400 python scripts/compare_fits.py dump gpurun_out/r_cur.npz
step r_compare 120 python scripts/compare_fits.py compare gpurun_out/r_prev.npz gpurun_out/r_cur.npz
rm -f gpurun_out/r_prev.npz gpurun_out/r_cur.npz
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2; do
  REDCLIFF_HIP_LIB=scripts/bin/lib_h.so step r_grid_h_$i 300 python bench.py $GR
  step r_grid_ch4_$i 300 python bench.py $GR
  REDCLIFF_HIP_LIB=scripts/bin/lib_prep2.so step r_grid_ch2_$i 300 python bench.py $GR
  REDCLIFF_HIP_LIB=scripts/bin/lib_prep1.so step r_grid_ch1_$i 300 python bench.py $GR
done
REDCLIFF_FORK=0 step r_trace 300 python scripts/phase_trace_pack.py --replicas 128 --steps 6
