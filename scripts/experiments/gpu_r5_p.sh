#!/bin/bash
# Round 5: defaults now 200-column embedder-forward slices and kernel-completed fork / join events;
# k_emb_final's adjacency workgroup in the combine launch (REDCLIFF_ADJ_EARLY): bitwise tests, A/B,
# per-step timeline; GPU suite + smoke on the defaults
source "$(dirname "$0")/../gpu_steps.sh"
step p_tests 600 python -u -m pytest tests/test_gpu_forked.py -v --timeout 300 --timeout-method thread -rA
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
  for cfg in c1k4 c4; do
    step p_${cfg}_base_$rep 200 $B --config $cfg
    REDCLIFF_ADJ_EARLY=1 step p_${cfg}_adj_$rep 200 $B --config $cfg
    REDCLIFF_EXT_EVENT=0 step p_${cfg}_noext_$rep 200 $B --config $cfg
  done
done
K="--steps 50 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times --config c1k4 --preheat-s 0"
REDCLIFF_ADJ_EARLY=1 step p_kt 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/p/kt -o run -- python bench.py $K
f=$(ls gpurun_out/p/kt/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && step p_timeline 60 python scripts/step_timeline.py "$f" --steps 4
rm -rf gpurun_out/p/kt
step p_suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA --durations=10
step p_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
