#!/bin/bash
# Round 5: GEMM epilogue operand loads issued together (dZ's mask), wave core at <= 5 waves' registers,
# plus the head / dhead load batching: bitwise whole packed fits against the previous build
# (scripts/bin/lib_prev.so), grid step A/B, per-kernel traces of both builds, GPU GEMM / pack tests.
source "$(dirname "$0")/../gpu_steps.sh"
P=scripts/bin/lib_prev.so
step av_tests 400 python -u -m pytest tests/test_gpu_generic.py tests/test_gpu_large_pack.py tests/test_gpu_replicas.py -x -q --timeout 150 --timeout-method thread
REDCLIFF_EMB_PATH=gemm COMPARE_FITS_R=32 REDCLIFF_HIP_LIB=$P step av_dump_prev 300 python scripts/compare_fits.py dump gpurun_out/av_prev.npz
REDCLIFF_EMB_PATH=gemm COMPARE_FITS_R=32 step av_dump_cur 300 python scripts/compare_fits.py dump gpurun_out/av_cur.npz
step av_cmp 120 python scripts/compare_fits.py compare gpurun_out/av_prev.npz gpurun_out/av_cur.npz
rm -f gpurun_out/av_*.npz
G="python scripts/grid_step.py --replicas 128 --steps 50"
for i in 1 2; do
  REDCLIFF_FORK=0 REDCLIFF_HIP_LIB=$P step av_g1_prev_$i 200 $G
  REDCLIFF_FORK=0 step av_g1_cur_$i 200 $G
  REDCLIFF_HIP_LIB=$P step av_gf_prev_$i 200 $G
  step av_gf_cur_$i 200 $G
done
REDCLIFF_HIP_LIB=$P REDCLIFF_FORK=0 step av_tr_prev 240 timeout -s KILL 220 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/av/prev -o run -- python scripts/grid_step.py --replicas 128 --steps 20
REDCLIFF_FORK=0 step av_tr_cur 240 timeout -s KILL 220 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/av/cur -o run -- python scripts/grid_step.py --replicas 128 --steps 20
for v in prev cur; do
  f=$(ls gpurun_out/av/$v/*/run_kernel_trace.csv gpurun_out/av/$v/run_kernel_trace.csv 2>/dev/null | head -n 1)
  python scripts/gemm_products.py "$f" --match k_ > gpurun_out/av_${v}_all.txt 2>&1
  rm -f "$f"
done
