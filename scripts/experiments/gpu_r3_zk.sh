#!/bin/bash
# Round 3: fc1 weight buffers in a column pairs per lane (float2 loads) -- A/B against the committed build
# (scripts/bin/lib_head.so), interleaved; forward / replica / autograd tests; TST timeline
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
B="python bench.py --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0"
for cfg in c4 c1k4 d4ic; do
  step zk_head_$cfg 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_head.so $B --config $cfg
  step zk_rot_$cfg 200 $B --config $cfg
done
step zk_trace_c4 200 python -u scripts/phase_trace.py --config c4
step zk_tests 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread
kill $HB
