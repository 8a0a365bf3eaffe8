#!/bin/bash
# Round 5: the wave GEMM core (k_rc_gemm_wave, REDCLIFF_GEMM_CORE=wave) against the LDS-tiled matrix
# core: bitwise (GEMM unit test, whole packed fits on the GEMM embedder), R = 128 grid step timing
# (one stream, alternating), per-product kernel trace.
source "$(dirname "$0")/../gpu_steps.sh"
step ar_unit 200 python -u -m pytest tests/test_gpu_generic.py -k gemm_cores -x -q --timeout 150 --timeout-method thread
for core in mfma wave; do
  REDCLIFF_EMB_PATH=gemm COMPARE_FITS_R=32 REDCLIFF_GEMM_CORE=$core step ar_dump_$core 300 python scripts/compare_fits.py dump gpurun_out/ar_fits_$core.npz
done
step ar_cmp 120 python scripts/compare_fits.py compare gpurun_out/ar_fits_mfma.npz gpurun_out/ar_fits_wave.npz
rm -f gpurun_out/ar_fits_*.npz
G="python scripts/grid_step.py --replicas 128 --steps 50"
for i in 1 2; do
  for core in mfma wave; do
    REDCLIFF_FORK=0 REDCLIFF_GEMM_CORE=$core step ar_g_${core}_$i 200 $G
  done
done
REDCLIFF_GEMM_CORE=wave step ar_gfork_wave 200 $G
REDCLIFF_GEMM_CORE=mfma step ar_gfork_mfma 200 $G
REDCLIFF_FORK=0 REDCLIFF_GEMM_CORE=wave step ar_tr_wave 240 timeout -s KILL 220 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ar/wave -o run -- python scripts/grid_step.py --replicas 128 --steps 20
f=$(ls gpurun_out/ar/wave/*/run_kernel_trace.csv gpurun_out/ar/wave/run_kernel_trace.csv 2>/dev/null | head -n 1)
python scripts/gemm_products.py "$f" > gpurun_out/ar_wave_products.txt 2>&1
python scripts/gemm_products.py "$f" --match k_ > gpurun_out/ar_wave_all.txt 2>&1
rm -f "$f"
