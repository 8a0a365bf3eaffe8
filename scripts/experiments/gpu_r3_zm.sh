#!/bin/bash
# Round 3: k_emb_tail (combine + embedder optimizer in one launch) -- bitwise tests first, then
# A/B via REDCLIFF_TAIL (interleaved), D4IC timeline, full GPU suite
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step zm_fork 300 python -u -m pytest tests/test_gpu_forked.py -v --timeout 120 --timeout-method thread
B="python bench.py --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0"
for cfg in d4ic c1k4 c4; do
  step zm_off_$cfg 200 env REDCLIFF_TAIL=0 $B --config $cfg
  step zm_on_$cfg 200 $B --config $cfg
done
step zm_off2_d4ic 200 env REDCLIFF_TAIL=0 $B --config d4ic
step zm_on2_d4ic 200 $B --config d4ic
step zm_trace_d4ic 200 python -u scripts/phase_trace.py --config d4ic
step zm_suite 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --durations=5
kill $HB
