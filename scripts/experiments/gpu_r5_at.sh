#!/bin/bash
# Round 5: wave core with k-contiguous operands transposed through the wave's LDS tile (wave) against
# every operand straight into the lanes (wd) and the LDS-tiled workgroups (mfma): GEMM unit test,
# whole packed fits bitwise with every product on the wave core, per-product traces.
source "$(dirname "$0")/../gpu_steps.sh"
step at_unit 200 python -u -m pytest tests/test_gpu_generic.py -k gemm_cores -x -q --timeout 150 --timeout-method thread
for core in mfma wave; do
  REDCLIFF_EMB_PATH=gemm COMPARE_FITS_R=32 REDCLIFF_GEMM_CORE=$core step at_dump_$core 300 python scripts/compare_fits.py dump gpurun_out/at_fits_$core.npz
done
step at_cmp 120 python scripts/compare_fits.py compare gpurun_out/at_fits_mfma.npz gpurun_out/at_fits_wave.npz
rm -f gpurun_out/at_fits_*.npz
for core in wave wd mfma; do
  REDCLIFF_FORK=0 REDCLIFF_GEMM_CORE=$core step at_tr_$core 240 timeout -s KILL 220 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/at/$core -o run -- python scripts/grid_step.py --replicas 128 --steps 20
  f=$(ls gpurun_out/at/$core/*/run_kernel_trace.csv gpurun_out/at/$core/run_kernel_trace.csv 2>/dev/null | head -n 1)
  python scripts/gemm_products.py "$f" > gpurun_out/at_${core}_products.txt 2>&1
  rm -f "$f"
done
