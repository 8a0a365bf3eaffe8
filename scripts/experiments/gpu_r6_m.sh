#!/bin/bash
# Round 6: the role-split k_fac_bwd_s16r (REDCLIFF_S16_ROLES=1) against k_fac_bwd_s16 in the same
# library -- whole packed fits bitwise (compare_fits R = 8: D4IC / C1(K=4) / TST), the packed-fit and
# data-parallel GPU tests on the role-split kernel, the R = 128 grid A/B and its workgroup trace.
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_FITS_R=8 COMPARE_FITS_CFGS=d4ic,c1k4,c4
REDCLIFF_S16_ROLES=0 step m_dump_s16 300 python scripts/compare_fits.py dump gpurun_out/m_s16.npz
REDCLIFF_S16_ROLES=1 step m_dump_roles 300 python scripts/compare_fits.py dump gpurun_out/m_roles.npz
step m_compare 120 python scripts/compare_fits.py compare gpurun_out/m_s16.npz gpurun_out/m_roles.npz
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2; do
  REDCLIFF_S16_ROLES=0 step m_grid_s16_$i 300 python bench.py $GR
  REDCLIFF_S16_ROLES=1 step m_grid_roles_$i 300 python bench.py $GR
done
REDCLIFF_S16_ROLES=1 REDCLIFF_FORK=0 step m_trace 300 python scripts/phase_trace_pack.py --replicas 128 --steps 6
REDCLIFF_S16_ROLES=1 step m_pytest 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pack_fit.py tests/test_gpu_large_pack.py tests/test_gpu_data_parallel.py
rm -f gpurun_out/m_s16.npz gpurun_out/m_roles.npz
