#!/bin/bash
# Round 5: the TST single fit's step (BASELINE configs[3] shape): phase trace and per-step timelines,
# one factor-backward launch (default) and the split-lead step forced
source "$(dirname "$0")/../gpu_steps.sh"
step ab_trace 200 python scripts/phase_trace.py --config c4
K="--steps 50 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times --config c4 --preheat-s 0"
step ab_kt 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab/kt -o run -- python bench.py $K
f=$(ls gpurun_out/ab/kt/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && step ab_timeline 60 python scripts/step_timeline.py "$f" --steps 3
REDCLIFF_SPLIT_LEAD=1 step ab_kt1 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab/kt1 -o run -- python bench.py $K
f=$(ls gpurun_out/ab/kt1/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && step ab_timeline1 60 python scripts/step_timeline.py "$f" --steps 3
rm -rf gpurun_out/ab/kt gpurun_out/ab/kt1
