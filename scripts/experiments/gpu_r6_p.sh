#!/bin/bash
# Round 6: the short factor kernels with the linear tile's LDS only (64 NK4 floats per wave, not the
# padded tile's + 160) and the backward's epilogue columns kept out of registers (125 VGPRs at D4IC:
# 4 resident workgroups per CU for both kernels) -- packed fits bitwise against the round's previous
# build, the packed tests, and the R = 128 grid A/B (D4IC, C1(K=4), TST) against the last commit.
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_FITS_R=8 COMPARE_FITS_CFGS=d4ic,c1k4,c4
REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so step p_dump_prev 300 python scripts/compare_fits.py dump gpurun_out/p_prev.npz
step p_dump_cur 300 python scripts/compare_fits.py dump gpurun_out/p_cur.npz
step p_compare 120 python scripts/compare_fits.py compare gpurun_out/p_prev.npz gpurun_out/p_cur.npz
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for cfg in d4ic c1k4 c4 d4ic; do
  REDCLIFF_HIP_LIB=scripts/bin/lib_h.so step p_grid_h_$cfg 300 python bench.py $GR --config $cfg
  step p_grid_cur_$cfg 300 python bench.py $GR --config $cfg
done
step p_pytest 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "packed or mfma" tests/test_gpu_pack_fit.py tests/test_gpu_large_pack.py
rm -f gpurun_out/p_prev.npz gpurun_out/p_cur.npz
