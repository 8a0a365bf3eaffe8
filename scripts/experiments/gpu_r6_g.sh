#!/bin/bash
# Round 6: light head / adjacency-reduce launch (k_emb_head_dadj) -- the C5 / GEMM-embedder suites; C5
# with k_emb_final at 1 / 4 / 8 parameter elements per thread; the reference grids' eight shares under
# the time-model sharding (REF_GRID_COST, min-max runs).
source "$(dirname "$0")/../gpu_steps.sh"
step g_tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_generic.py tests/test_gpu_large_pack.py \
  tests/test_gpu_replicas.py -v --timeout 300 --timeout-method thread -rA \
  -k "stress or embgemm or packed or product_sets or pack_of_128 or validate or xcd or single_active" --durations=5
C5="--config c5 --no-cpu-baseline --steps 100 --warmup 10 --replicas 1 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2; do
  step g_c5_ept1_$i 300 python bench.py $C5
  REDCLIFF_EMB_FINAL_EPT=4 step g_c5_ept4_$i 300 python bench.py $C5
  REDCLIFF_EMB_FINAL_EPT=8 step g_c5_ept8_$i 300 python bench.py $C5
done
step g_refgrid_all 900 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --replicas 1 --fit-replicas 0 \
  --dp-leg-batch 0 --no-north-star --c5-steps 0 --ref-grid-all-shares
