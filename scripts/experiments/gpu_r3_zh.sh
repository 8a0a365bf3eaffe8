#!/bin/bash
# Round 3: fc1-weight L2 warm-up in the embedder forward -- A/B against FW_TOUCH=0 (interleaved),
# GPU suite, TST timeline
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
B="python bench.py --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0"
for cfg in c4 c1k4 d4ic; do
  step zh_off_$cfg 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_notouch.so $B --config $cfg
  step zh_on_$cfg 200 $B --config $cfg
done
step zh_off2_c1k4 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_notouch.so $B --config c1k4
step zh_on2_c1k4 200 $B --config c1k4
step zh_trace_c4 200 python -u scripts/phase_trace.py --config c4
step zh_suite 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --durations=5
kill $HB
