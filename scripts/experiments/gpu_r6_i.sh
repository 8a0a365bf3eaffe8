#!/bin/bash
# Round 6: k_emb_final as adjacency + parameter launches when its LDS is large (C5) -- bitwise test, the C5
# error-budget test, C5 A/B (REDCLIFF_EMB_FINAL_SPLIT=0/1) and its kernel stats.
source "$(dirname "$0")/../gpu_steps.sh"
step i_tests 600 python -u -m pytest tests/test_gpu_generic.py tests/test_gpu_parity.py -v --timeout 300 \
  --timeout-method thread -rA -k "emb_final_split or stress or product_sets"
C5="--config c5 --no-cpu-baseline --steps 100 --warmup 10 --replicas 1 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
for i in 1 2; do
  REDCLIFF_EMB_FINAL_SPLIT=0 step i_c5_split0_$i 300 python bench.py $C5
  REDCLIFF_EMB_FINAL_SPLIT=1 step i_c5_split1_$i 300 python bench.py $C5
done
step i_c5stats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/i/c5stats -o run -- python bench.py $C5 --no-kernel-times
rm -f gpurun_out/i/*/run_kernel_trace.csv
