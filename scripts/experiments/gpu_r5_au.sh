#!/bin/bash
# Round 5: packed-grid embedder head / dhead loads batched (k_lemb_head issued 68 serial load round trips
# per wave), LDS chains of the windowed kernels unrolled: bitwise whole packed fits against the previous
# build (scripts/bin/lib_prev.so), grid step A/B, per-kernel trace, GPU suite, bench line.
source "$(dirname "$0")/../gpu_steps.sh"
REDCLIFF_EMB_PATH=gemm COMPARE_FITS_R=32 REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so step au_dump_prev 300 python scripts/compare_fits.py dump gpurun_out/au_prev.npz
REDCLIFF_EMB_PATH=gemm COMPARE_FITS_R=32 step au_dump_cur 300 python scripts/compare_fits.py dump gpurun_out/au_cur.npz
step au_cmp 120 python scripts/compare_fits.py compare gpurun_out/au_prev.npz gpurun_out/au_cur.npz
rm -f gpurun_out/au_*.npz
G="python scripts/grid_step.py --replicas 128 --steps 50"
for i in 1 2; do
  REDCLIFF_FORK=0 REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so step au_g1_prev_$i 200 $G
  REDCLIFF_FORK=0 step au_g1_cur_$i 200 $G
  REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so step au_gf_prev_$i 200 $G
  step au_gf_cur_$i 200 $G
done
for v in prev cur; do
  L=""; [ $v = prev ] && L=scripts/bin/lib_prev.so
  REDCLIFF_HIP_LIB=$L REDCLIFF_FORK=0 step au_tr_$v 240 timeout -s KILL 220 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/au/$v -o run -- python scripts/grid_step.py --replicas 128 --steps 20
  f=$(ls gpurun_out/au/$v/*/run_kernel_trace.csv gpurun_out/au/$v/run_kernel_trace.csv 2>/dev/null | head -n 1)
  python scripts/gemm_products.py "$f" --match k_ > gpurun_out/au_${v}_all.txt 2>&1
  rm -f "$f"
done
step au_suite 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rA
step au_bench 600 python bench.py
