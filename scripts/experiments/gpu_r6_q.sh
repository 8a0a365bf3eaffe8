#!/bin/bash
# Round 6: the short factor kernels with the linear tile's LDS only (64 NK4 floats per wave, not the
# padded tile's + 160; the forward at D4IC then fits 5 workgroups per CU), the backward's registers as
# before -- packed fits bitwise against the round's previous build, the R = 128 grid A/B (D4IC twice,
# C1(K=4), TST) against the last commit.
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_FITS_R=8 COMPARE_FITS_CFGS=d4ic,c1k4,c4
REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so step q_dumq_prev 300 python scripts/compare_fits.py dump gpurun_out/q_prev.npz
step q_dumq_cur 300 python scripts/compare_fits.py dump gpurun_out/q_cur.npz
step q_compare 120 python scripts/compare_fits.py compare gpurun_out/q_prev.npz gpurun_out/q_cur.npz
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
i=0
for cfg in d4ic c1k4 c4 d4ic; do
  i=$((i+1))
  REDCLIFF_HIP_LIB=scripts/bin/lib_h.so step q_grid_h_${cfg}_$i 300 python bench.py $GR --config $cfg
  step q_grid_cur_${cfg}_$i 300 python bench.py $GR --config $cfg
done
rm -f gpurun_out/q_prev.npz gpurun_out/q_cur.npz
REDCLIFF_FORK=0 step q_trace 300 python scripts/phase_trace_pack.py --replicas 128 --steps 6
