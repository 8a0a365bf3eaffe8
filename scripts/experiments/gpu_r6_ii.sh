#!/bin/bash
# Round 6: k_lemb_dhead requesting fc2W / f1 / w / labels before its dL/dw sums (RC_DHEAD_EARLY=1)
# and k_lemb_gfc's window loop unrolled 32 times (RC_GFC_UNROLL=32), against the tree -- packed fits
# bitwise (R = 16: GEMM embedder) for both together, kernel-trace summaries per arm, R = 128 grid A/B.
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_FITS_R=16 COMPARE_FITS_CFGS=d4ic,c1k4,c4
step ii_dump_0 300 python scripts/compare_fits.py dump gpurun_out/ii_0.npz
REDCLIFF_HIP_LIB=scripts/bin/lib_dhgfc.so step ii_dump_1 300 python scripts/compare_fits.py dump gpurun_out/ii_1.npz
step ii_compare 120 python scripts/compare_fits.py compare gpurun_out/ii_0.npz gpurun_out/ii_1.npz
rm -f gpurun_out/ii_0.npz gpurun_out/ii_1.npz
for cfg in d4ic c4; do
  for v in tree dheadearly gfc32 dhgfc; do
    if [ $v = tree ]; then unset REDCLIFF_HIP_LIB; else export REDCLIFF_HIP_LIB=scripts/bin/lib_$v.so; fi
    REDCLIFF_FORK=0 step ii_stats_${v}_$cfg 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ii/${v}_$cfg -o run -- python scripts/grid_step.py --replicas 128 --steps 20 --config $cfg
  done
done
unset REDCLIFF_HIP_LIB
rm -f gpurun_out/ii/*/run_kernel_trace.csv
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2; do
  for cfg in c4 d4ic; do
    step ii_grid_0_${cfg}_$i 300 python bench.py $GR --config $cfg
    REDCLIFF_HIP_LIB=scripts/bin/lib_dhgfc.so step ii_grid_1_${cfg}_$i 300 python bench.py $GR --config $cfg
  done
done
