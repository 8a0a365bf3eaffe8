#!/bin/bash
# Round 5: the split-lead step on one stream (REDCLIFF_SPLIT_ONE=1: lead launch, then the embedder
# backward and the factor update in one launch, k_emb_bwd_upd at 3 waves per SIMD) against the
# two-stream split-lead step: bitwise test, C1(K=4) / TST A/B, per-step timeline
source "$(dirname "$0")/../gpu_steps.sh"
step v_tests 600 python -u -m pytest tests/test_gpu_forked.py -v --timeout 300 --timeout-method thread -rA
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
  for cfg in c1k4 c4; do
    step v_${cfg}_base_$rep 200 $B --config $cfg
    REDCLIFF_SPLIT_ONE=1 step v_${cfg}_one_$rep 200 $B --config $cfg
    REDCLIFF_SPLIT_ONE=1 REDCLIFF_SPLIT_LEAD=1 step v_${cfg}_one_forced_$rep 200 $B --config $cfg
  done
done
K="--steps 50 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times --config c1k4 --preheat-s 0"
REDCLIFF_SPLIT_ONE=1 step v_kt 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/v/kt -o run -- python bench.py $K
f=$(ls gpurun_out/v/kt/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && step v_timeline 60 python scripts/step_timeline.py "$f" --steps 4
rm -rf gpurun_out/v/kt
