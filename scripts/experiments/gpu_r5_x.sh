#!/bin/bash
# Round 5: where the packed fit's wall clock beyond its training steps goes (fits/hour leg shape:
# D4IC, R = 128, 40 epochs, 8 training + 2 validation batches): the host split per epoch, the
# wrapped-section times, and a kernel trace's busy / idle split
source "$(dirname "$0")/../gpu_steps.sh"
step x_prof 300 python scripts/pack_fit_profile.py --replicas 128 --epochs 40 --host-split
step x_kt 300 timeout -s KILL 280 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/x/kt -o run -- python scripts/pack_fit_profile.py --replicas 128 --epochs 40
f=$(ls gpurun_out/x/kt/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && step x_gaps 120 python scripts/trace_gaps.py "$f" --split-ms 20 --top 30
rm -rf gpurun_out/x/kt
