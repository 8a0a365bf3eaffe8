#!/bin/bash
# Round 6: which role bounds k_fac_bwd_s16r -- timing-only builds with the update waves idle
# (RC_S16_EXP=4) or the contract waves idle (8), barriers kept; the R = 128 grid leg each.
source "$(dirname "$0")/../gpu_steps.sh"
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
REDCLIFF_S16_ROLES=1 step n_grid_roles 300 python bench.py $GR
for v in 4 8; do
  REDCLIFF_HIP_LIB=scripts/bin/lib_s16rexp$v.so step n_grid_rexp$v 300 python bench.py $GR
done
