#!/bin/bash
# Round 6: product sets on the wave core (packed grids) and the merged dS / BatchNorm ends -- bitwise
# tests; C5 and the R = 128 grid A/B (REDCLIFF_GEMM_SET=0/1), C5 with 32 x 32 set tiles.
source "$(dirname "$0")/../gpu_steps.sh"
step d_tests 600 python -u -m pytest tests/test_gpu_generic.py tests/test_gpu_large_pack.py -v --timeout 300 \
  --timeout-method thread -rA -k "product_sets or cores_bitwise or pack_of_128 or forked_pack"
C5="--config c5 --no-cpu-baseline --steps 100 --warmup 10 --replicas 1 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2; do
  REDCLIFF_GEMM_SET=0 step d_c5_set0_$i 300 python bench.py $C5
  REDCLIFF_GEMM_SET=1 step d_c5_set1_$i 300 python bench.py $C5
  REDCLIFF_GEMM_SET=1 REDCLIFF_GEMM_TILE=32 step d_c5_set1_t32_$i 300 python bench.py $C5
  REDCLIFF_GEMM_SET=0 step d_grid_set0_$i 300 python bench.py $GR
  REDCLIFF_GEMM_SET=1 step d_grid_set1_$i 300 python bench.py $GR
done
