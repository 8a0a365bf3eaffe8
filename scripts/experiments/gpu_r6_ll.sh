#!/bin/bash
# Round 6: TST's k_emb_final_params with the register allocator held to 4 / 5 waves per SIMD
# (RC_EF_PARAMS_WAVES; the tree's choice is 152 VGPRs, 3 waves) -- kernel-trace summaries of the
# R = 128 TST grid per arm, packed fits bitwise for the 4-wave arm (R = 16, TST).
source "$(dirname "$0")/../gpu_steps.sh"
for v in tree efw4 efw5; do
  if [ $v = tree ]; then unset REDCLIFF_HIP_LIB; else export REDCLIFF_HIP_LIB=scripts/bin/lib_$v.so; fi
  REDCLIFF_FORK=0 step ll_stats_$v 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ll/$v -o run -- python scripts/grid_step.py --replicas 128 --steps 20 --config c4
done
unset REDCLIFF_HIP_LIB
rm -f gpurun_out/ll/*/run_kernel_trace.csv
export COMPARE_FITS_R=16 COMPARE_FITS_CFGS=c4
step ll_dump_0 300 python scripts/compare_fits.py dump gpurun_out/ll_0.npz
REDCLIFF_HIP_LIB=scripts/bin/lib_efw4.so step ll_dump_1 300 python scripts/compare_fits.py dump gpurun_out/ll_1.npz
step ll_compare 120 python scripts/compare_fits.py compare gpurun_out/ll_0.npz gpurun_out/ll_1.npz
rm -f gpurun_out/ll_0.npz gpurun_out/ll_1.npz
