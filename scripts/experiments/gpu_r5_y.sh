#!/bin/bash
# Round 5, timing-only experiment (the variants compute WRONG results): what the split-lead step's
# cross-stream hand-offs cost at C1(K=4) -- the update launched without its fork wait
# (lib_nofork.so), without the join before k_emb_final (lib_nojoin.so), without both (lib_noboth.so)
source "$(dirname "$0")/../gpu_steps.sh"
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times --config c1k4"
for rep in 1 2; do
  step y_base_$rep 200 $B
  for v in nofork nojoin noboth; do
    REDCLIFF_HIP_LIB=scripts/bin/lib_$v.so step y_${v}_$rep 200 $B
  done
done
K="--steps 50 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times --config c1k4 --preheat-s 0"
REDCLIFF_HIP_LIB=scripts/bin/lib_nofork.so step y_kt 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/y/kt -o run -- python bench.py $K
f=$(ls gpurun_out/y/kt/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && step y_timeline 60 python scripts/step_timeline.py "$f" --steps 4
rm -rf gpurun_out/y/kt
