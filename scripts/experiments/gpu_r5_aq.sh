#!/bin/bash
# Round 5: the R = 128 grid's embedder GEMM products: tile 64 / 32 x operand K steps in flight
# (REDCLIFF_GEMM_PD = 1 / 2 / 3), one stream; bitwise check of PD = 2 / 3 against PD = 1 on whole
# packed fits (GEMM embedder); per-product kernel traces of the two leading candidates.
source "$(dirname "$0")/../gpu_steps.sh"
G="python scripts/grid_step.py --replicas 128 --steps 20"
for t in 64 32; do
  for pd in 1 2 3; do
    REDCLIFF_FORK=0 REDCLIFF_GEMM_TILE=$t REDCLIFF_GEMM_PD=$pd step aq_t${t}_pd$pd 200 $G
  done
done
for pd in 1 2 3; do
  REDCLIFF_EMB_PATH=gemm COMPARE_FITS_R=32 REDCLIFF_GEMM_PD=$pd step aq_dump_pd$pd 300 python scripts/compare_fits.py dump gpurun_out/aq_fits_pd$pd.npz
done
step aq_cmp2 120 python scripts/compare_fits.py compare gpurun_out/aq_fits_pd1.npz gpurun_out/aq_fits_pd2.npz
step aq_cmp3 120 python scripts/compare_fits.py compare gpurun_out/aq_fits_pd1.npz gpurun_out/aq_fits_pd3.npz
rm -f gpurun_out/aq_fits_pd*.npz
for v in 64:1 64:2 32:2; do
  t=${v%:*}; pd=${v#*:}
  REDCLIFF_FORK=0 REDCLIFF_GEMM_TILE=$t REDCLIFF_GEMM_PD=$pd step aq_tr_t${t}_pd$pd 240 timeout -s KILL 220 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/aq/t${t}_pd$pd -o run -- $G
  f=$(ls gpurun_out/aq/t${t}_pd$pd/*/run_kernel_trace.csv gpurun_out/aq/t${t}_pd$pd/run_kernel_trace.csv 2>/dev/null | head -n 1)
  python scripts/gemm_products.py "$f" > gpurun_out/aq_t${t}_pd${pd}_products.txt 2>&1
  python scripts/gemm_products.py "$f" --match k_ > gpurun_out/aq_t${t}_pd${pd}_all.txt 2>&1
  rm -f "$f"
done
