#!/bin/bash
# Round 6: product sets (independent GEMM-embedder products in one launch) -- bitwise tests, the C5
# A/B and its kernel trace.
source "$(dirname "$0")/../gpu_steps.sh"
step b_tests 600 python -u -m pytest tests/test_gpu_generic.py -v --timeout 300 --timeout-method thread -rA \
  -k "product_sets or cores_bitwise or hip_adam_reloaded"
C5="--config c5 --no-cpu-baseline --steps 100 --warmup 10 --replicas 1 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2; do
  REDCLIFF_GEMM_SET=0 step b_c5_set0_$i 300 python bench.py $C5
  REDCLIFF_GEMM_SET=1 step b_c5_set1_$i 300 python bench.py $C5
done
step b_c5_kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b_c5_kt -o run -- python bench.py $C5 --no-kernel-times
