#!/bin/bash
# Round 5: GPU suite + smoke on the new defaults (channel-sliced embedder forward, fence-free fork /
# join events, 3-wave k_fac_bwd_s16); per-step kernel timelines of C1(K=4) with and without the split
# lead; the default bench line
source "$(dirname "$0")/../gpu_steps.sh"
step n_suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA --durations=10
step n_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
K="--steps 50 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times --config c1k4 --preheat-s 0"
step n_kt 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/n/kt -o run -- python bench.py $K
f=$(ls gpurun_out/n/kt/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && step n_timeline 60 python scripts/step_timeline.py "$f" --steps 4
REDCLIFF_SPLIT_LEAD=0 step n_kt0 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/n/kt0 -o run -- python bench.py $K
f=$(ls gpurun_out/n/kt0/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && step n_timeline0 60 python scripts/step_timeline.py "$f" --steps 4
rm -rf gpurun_out/n/kt gpurun_out/n/kt0
step n_bench 600 python bench.py
