#!/bin/bash
# Round 3: embedder-backward staging variants at TST / C1(K=4) (none, dL/dw rounds together, BN
# staging, both = default), interleaved twice
source "$(dirname "$0")/../gpu_steps.sh"
B="python bench.py --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0"
for rep in 1 2; do
  for v in none dw bn; do
    step zg_${v}_c4_$rep 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_$v.so $B --config c4
  done
  step zg_both_c4_$rep 200 $B --config c4
done
for v in none dw bn; do
  step zg_${v}_c1k4 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_$v.so $B --config c1k4
done
step zg_both_c1k4 200 $B --config c1k4
