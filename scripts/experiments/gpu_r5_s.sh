#!/bin/bash
# Round 5: fc1 of a one-window embedder-forward workgroup with all four column steps of its slice
# requested before the graph convolution (scripts/bin/lib_all4w3.so: 139 VGPRs, 3 waves; lib_all4w4.so:
# forced to 4 waves, 36 bytes of scratch) against the current build, single fits C1(K=4) / TST / D4IC
source "$(dirname "$0")/../gpu_steps.sh"
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
  for cfg in c1k4 c4 d4ic; do
    step s_${cfg}_base_$rep 200 $B --config $cfg
    REDCLIFF_HIP_LIB=scripts/bin/lib_all4w3.so step s_${cfg}_w3_$rep 200 $B --config $cfg
    REDCLIFF_HIP_LIB=scripts/bin/lib_all4w4.so step s_${cfg}_w4_$rep 200 $B --config $cfg
  done
done
REDCLIFF_HIP_LIB=scripts/bin/lib_all4w3.so step s_tests 600 python -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -rA
