#!/bin/bash
# Round 5: (1) run-to-run determinism of the small synthetic-grid shapes (K, p) = (2, 3), (1, 12) on the
# packed-grid kernels, isolating the factor (mfma / vector) and embedder (gemm / fused) paths and the
# fork; (2) the failing tests; (3) the GEMM-embedder small-kernel load changes: bitwise whole packed
# fits previous vs current build, and R = 128 grid-step kernel times
source "$(dirname "$0")/../gpu_steps.sh"
P=scripts/bin/lib_prev_r5i.so
S="--shapes 2x3,1x12"
REDCLIFF_FAC_PATH=mfma REDCLIFF_EMB_PATH=gemm step i_det_mg 300 python -u scripts/determinism_probe.py $S
REDCLIFF_FAC_PATH=mfma REDCLIFF_EMB_PATH=fused step i_det_mf 300 python -u scripts/determinism_probe.py $S
REDCLIFF_FAC_PATH=vector REDCLIFF_EMB_PATH=gemm step i_det_vg 300 python -u scripts/determinism_probe.py $S
REDCLIFF_FORK=0 REDCLIFF_FAC_PATH=mfma REDCLIFF_EMB_PATH=gemm step i_det_mg_nofork 300 python -u scripts/determinism_probe.py $S
REDCLIFF_FAC_PATH=mfma REDCLIFF_EMB_PATH=gemm step i_det_mg_steps 300 python -u scripts/determinism_probe.py $S --steps-only
step i_tests 600 python -u -m pytest tests/test_gpu_generic.py tests/test_gpu_pack_fit.py -v --timeout 300 --timeout-method thread -rA
for R in 4 32; do
  COMPARE_FITS_R=$R REDCLIFF_EMB_PATH=gemm REDCLIFF_HIP_LIB=$P step i_dump_prev_$R 300 python scripts/compare_fits.py dump gpurun_out/fprev_$R.npz
  COMPARE_FITS_R=$R REDCLIFF_EMB_PATH=gemm step i_dump_cur_$R 300 python scripts/compare_fits.py dump gpurun_out/fcur_$R.npz
  step i_cmp_$R 60 python scripts/compare_fits.py compare gpurun_out/fprev_$R.npz gpurun_out/fcur_$R.npz
done
rm -f gpurun_out/fprev_*.npz gpurun_out/fcur_*.npz
REDCLIFF_HIP_LIB=$P step i_sweep_prev 400 python scripts/grid_sweep.py --replicas 128 --steps 30 --rounds 2 --kernel-times --settings '[{"REDCLIFF_FORK":"0"}]'
step i_sweep_cur 400 python scripts/grid_sweep.py --replicas 128 --steps 30 --rounds 2 --kernel-times --settings '[{"REDCLIFF_FORK":"0"}]'
