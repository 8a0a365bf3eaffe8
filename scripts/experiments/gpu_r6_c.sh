#!/bin/bash
# Round 6: the reference grids' eight shares (TST and synthetic), timed one after another on one GPU.
source "$(dirname "$0")/../gpu_steps.sh"
step c_refgrid_all 1100 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --replicas 1 --fit-replicas 0 \
  --dp-leg-batch 0 --no-north-star --c5-steps 0 --ref-grid-all-shares
