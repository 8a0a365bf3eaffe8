#!/bin/bash
# Round 5: D4IC single fit (the bench line's value): phase trace of the fused step and the per-step kernel
# timeline from a rocprofv3 kernel trace; C1(K=4) phase trace on the current defaults
source "$(dirname "$0")/../gpu_steps.sh"
step r_trace_d4ic 200 python scripts/phase_trace.py --config d4ic
step r_trace_c1k4 200 python scripts/phase_trace.py --config c1k4
K="--steps 50 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times --preheat-s 0"
step r_kt 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r/kt -o run -- python bench.py $K --config d4ic
f=$(ls gpurun_out/r/kt/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && step r_timeline 60 python scripts/step_timeline.py "$f" --steps 4
rm -rf gpurun_out/r/kt
