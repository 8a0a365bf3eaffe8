#!/bin/bash
# Round 6: parameter elements per thread of TST's split k_emb_final_params (REDCLIFF_EMB_FINAL_EPT
# 2 / 4 / 8; 8 is the default from 96 replicas) -- kernel-trace summaries and R = 128 grid A/B.
source "$(dirname "$0")/../gpu_steps.sh"
for e in 8 4 2; do
  REDCLIFF_EMB_FINAL_EPT=$e REDCLIFF_FORK=0 step jj_stats_$e 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/jj/$e -o run -- python scripts/grid_step.py --replicas 128 --steps 20 --config c4
done
rm -f gpurun_out/jj/*/run_kernel_trace.csv
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0 --config c4"
for i in 1 2; do
  for e in 8 4 2; do
    REDCLIFF_EMB_FINAL_EPT=$e step jj_grid_${e}_$i 300 python bench.py $GR
  done
done
