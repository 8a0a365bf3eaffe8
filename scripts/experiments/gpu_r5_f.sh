#!/bin/bash
# Round 5: (1) fit_packs + packed-fit tests, (2) bitwise: the previous build (scripts/bin/lib_prev_r5.so)
# against the current one (reciprocal-form Adam divisions) on whole packed fits at R = 1 / 4 / 8 / 32,
# (3) the reference-grid leg with concurrent packs, (4) k_fac_bwd_s16 per-kernel times: previous vs
# current build, and the stagger knob
source "$(dirname "$0")/../gpu_steps.sh"
P=scripts/bin/lib_prev_r5.so
step f_tests 600 python -u -m pytest tests/test_gpu_pack_fit.py tests/test_gpu_replicas.py tests/test_gpu_large_pack.py -v --timeout 300 --timeout-method thread -rA
for R in 1 4 8 32; do
  COMPARE_FITS_R=$R REDCLIFF_HIP_LIB=$P step f_dump_prev_$R 300 python scripts/compare_fits.py dump gpurun_out/fprev_$R.npz
  COMPARE_FITS_R=$R step f_dump_cur_$R 300 python scripts/compare_fits.py dump gpurun_out/fcur_$R.npz
  step f_cmp_$R 60 python scripts/compare_fits.py compare gpurun_out/fprev_$R.npz gpurun_out/fcur_$R.npz
done
rm -f gpurun_out/fprev_*.npz gpurun_out/fcur_*.npz
step f_refgrid 600 python bench.py --steps 5 --warmup 2 --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --no-cpu-baseline --no-north-star --no-kernel-times
REDCLIFF_HIP_LIB=$P step f_sweep_prev 400 python scripts/grid_sweep.py --replicas 128 --steps 30 --rounds 2 --kernel-times --settings '[{"REDCLIFF_FORK":"0"}]'
step f_sweep_cur 600 python scripts/grid_sweep.py --replicas 128 --steps 30 --rounds 2 --kernel-times --settings '[{"REDCLIFF_FORK":"0"},{"REDCLIFF_FORK":"0","REDCLIFF_S16_STAGGER":"1"},{"REDCLIFF_FORK":"0","REDCLIFF_S16_STAGGER":"2"},{"REDCLIFF_FORK":"0","REDCLIFF_S16_STAGGER":"1:odd"},{"REDCLIFF_FORK":"0","REDCLIFF_S16_STAGGER":"1:prio"},{"REDCLIFF_FORK":"0","REDCLIFF_S16_STAGGER":"1:odd:prio"}]'
