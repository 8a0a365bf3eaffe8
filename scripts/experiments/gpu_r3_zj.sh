#!/bin/bash
# Round 3: fc1 weight buffers in a move-free rotation, one accumulator column per window at SB = 1 -- A/B against the committed build
# (scripts/bin/lib_head.so), interleaved; forward / replica / autograd tests; TST timeline
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
B="python bench.py --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0"
for cfg in c4 c1k4 d4ic; do
  step zj_head_$cfg 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_head.so $B --config $cfg
  step zj_rot_$cfg 200 $B --config $cfg
done
step zj_trace_c4 200 python -u scripts/phase_trace.py --config c4
step zj_tests 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread
kill $HB
