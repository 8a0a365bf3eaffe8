#!/bin/bash
# Round 6: k_fac_fwd_s16's blocks per wave (REDCLIFF_FAC_BPW_FWD; default: about two rounds of resident
# workgroups) on the R = 128 grid, D4IC and TST.
source "$(dirname "$0")/../gpu_steps.sh"
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0"
step s_grid_def_a 300 python bench.py $GR
for b in 3 4 6 7 9 12; do
  REDCLIFF_FAC_BPW_FWD=$b step s_grid_bpw$b 300 python bench.py $GR
done
step s_grid_def_b 300 python bench.py $GR
step s_grid_c4_def 300 python bench.py $GR --config c4
for b in 3 6 8; do
  REDCLIFF_FAC_BPW_FWD=$b step s_grid_c4_bpw$b 300 python bench.py $GR --config c4
done
