#!/bin/bash
# Round 6: k_fac_bwd_s16 over 16-unit blocks of the replica's K*p*h (blocks may span two networks;
# the networks' adjacency rows staged once per workgroup) -- whole packed fits bitwise against the
# round's previous build (compare_fits R = 8: D4IC h = 100, C1(K=4) / TST h = 25), the unit-block
# parity tests and the packed-fit tests, and the R = 128 grid A/B against the last commit's library.
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_FITS_R=8 COMPARE_FITS_CFGS=d4ic,c1k4,c4
REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so step o_dump_prev 300 python scripts/compare_fits.py dump gpurun_out/o_prev.npz
step o_dump_cur 300 python scripts/compare_fits.py dump gpurun_out/o_cur.npz
step o_compare 120 python scripts/compare_fits.py compare gpurun_out/o_prev.npz gpurun_out/o_cur.npz
REDCLIFF_HIP_LIB=scripts/bin/lib_h.so step o_pytest_h12_prev 300 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "unit_blocks"
step o_pytest 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "unit_blocks or packed or mfma" tests/test_gpu_pack_fit.py tests/test_gpu_large_pack.py
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2; do
  REDCLIFF_HIP_LIB=scripts/bin/lib_h.so step o_grid_h_$i 300 python bench.py $GR
  step o_grid_cur_$i 300 python bench.py $GR
done
for cfg in c1k4 c4; do
  REDCLIFF_HIP_LIB=scripts/bin/lib_h.so step o_grid_h_$cfg 300 python bench.py $GR --config $cfg
  step o_grid_cur_$cfg 300 python bench.py $GR --config $cfg
done
rm -f gpurun_out/o_prev.npz gpurun_out/o_cur.npz
