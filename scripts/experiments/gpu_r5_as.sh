#!/bin/bash
# Round 5: the wave GEMM core as the default for m/n-contiguous products: GEMM + embedder suites,
# bitwise whole packed fits against the LDS core, grid step A/B (one stream and forked), per-product
# trace, the bench line.
source "$(dirname "$0")/../gpu_steps.sh"
step as_tests 400 python -u -m pytest tests/test_gpu_generic.py tests/test_gpu_large_pack.py tests/test_gpu_replicas.py -x -q --timeout 150 --timeout-method thread
for core in mfma def; do
  if [ $core = def ]; then unset REDCLIFF_GEMM_CORE; else export REDCLIFF_GEMM_CORE=$core; fi
  REDCLIFF_EMB_PATH=gemm COMPARE_FITS_R=32 step as_dump_$core 300 python scripts/compare_fits.py dump gpurun_out/as_fits_$core.npz
done
unset REDCLIFF_GEMM_CORE
step as_cmp 120 python scripts/compare_fits.py compare gpurun_out/as_fits_mfma.npz gpurun_out/as_fits_def.npz
rm -f gpurun_out/as_fits_*.npz
G="python scripts/grid_step.py --replicas 128 --steps 50"
for i in 1 2; do
  REDCLIFF_FORK=0 REDCLIFF_GEMM_CORE=mfma step as_g1_mfma_$i 200 $G
  REDCLIFF_FORK=0 step as_g1_def_$i 200 $G
  REDCLIFF_GEMM_CORE=mfma step as_gf_mfma_$i 200 $G
  step as_gf_def_$i 200 $G
done
REDCLIFF_FORK=0 step as_tr 240 timeout -s KILL 220 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/as/def -o run -- python scripts/grid_step.py --replicas 128 --steps 20
f=$(ls gpurun_out/as/def/*/run_kernel_trace.csv gpurun_out/as/def/run_kernel_trace.csv 2>/dev/null | head -n 1)
python scripts/gemm_products.py "$f" > gpurun_out/as_def_products.txt 2>&1
python scripts/gemm_products.py "$f" --match k_ > gpurun_out/as_def_all.txt 2>&1
rm -f "$f"
step as_bench 600 python bench.py
