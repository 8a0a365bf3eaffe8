#!/bin/bash
# Round 6: the reference grids' eight shares, round-5 FLOP-weighted cut against the time-model cut,
# back to back on one box.
source "$(dirname "$0")/../gpu_steps.sh"
A="python bench.py --no-cpu-baseline --steps 20 --warmup 5 --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --no-north-star --c5-steps 0 --ref-grid-all-shares"
step h_old_1 560 $A --ref-grid-model 0
step h_model_1 560 $A --ref-grid-model 1
