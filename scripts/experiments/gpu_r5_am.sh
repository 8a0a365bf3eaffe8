#!/bin/bash
# Round 5: the bench's data-parallel leg read 1.31 M windows/s at r5t and 0.98 M at r5u.  Same box:
# the current build with sharded / whole-set storage, and the session-start build
# (scripts/bin/lib_start_r5s.so, cfcd5d1's csrc) with sharded storage.
source "$(dirname "$0")/../gpu_steps.sh"
D="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
  step am_cur_$rep 200 $D
  REDCLIFF_DP_SHARDED=0 step am_whole_$rep 200 $D
  REDCLIFF_HIP_LIB=scripts/bin/lib_start_r5s.so step am_start_$rep 200 $D
done
