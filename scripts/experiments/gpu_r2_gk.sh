#!/bin/bash
# Round 2: GEMM K-step depth (RC_GEMM_K = 16 / 32 / 64, same in-order k chain) at C5, with the
# bitwise core test on each variant library.
source "$(dirname "$0")/../gpu_steps.sh"
C5="python -u bench.py --config c5 --steps 30 --warmup 5 --replicas 1 --fit-replicas 0 --no-cpu-baseline --no-north-star --no-kernel-times"
step gk16 300 $C5
for k in 32 64; do
  REDCLIFF_HIP_LIB=$PWD/scripts/bin/lib_gk$k.so step gk${k}_test 300 python -u -m pytest tests/test_gpu_generic.py -k "gemm" -v --timeout 200 --timeout-method thread
  REDCLIFF_HIP_LIB=$PWD/scripts/bin/lib_gk$k.so step gk$k 300 $C5
done
