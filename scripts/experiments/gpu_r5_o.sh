#!/bin/bash
# Round 5: GPU suite + smoke on the current defaults (channel-sliced embedder forward, fence-free fork /
# join events, 3-wave k_fac_bwd_s16); fork / join events completed by the kernels themselves
# (REDCLIFF_EXT_EVENT=1) on the single fits, with per-step kernel timelines; the default bench line
source "$(dirname "$0")/../gpu_steps.sh"
step o_suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA --durations=10
step o_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
K="--steps 50 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times --config c1k4 --preheat-s 0"
REDCLIFF_EXT_EVENT=1 step o_kt 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/o/kt -o run -- python bench.py $K
f=$(ls gpurun_out/o/kt/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && step o_timeline_ext 60 python scripts/step_timeline.py "$f" --steps 4
rm -rf gpurun_out/o/kt
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
  for cfg in c1k4 c4; do
    step o_${cfg}_base_$rep 200 $B --config $cfg
    REDCLIFF_EXT_EVENT=1 step o_${cfg}_ext_$rep 200 $B --config $cfg
  done
done
REDCLIFF_EXT_EVENT=1 step o_ext_tests 600 python -u -m pytest tests/test_gpu_forked.py tests/test_gpu_fit_golden.py -v --timeout 300 --timeout-method thread -rA
step o_bench 600 python bench.py
