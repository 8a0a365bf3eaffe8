#!/bin/bash
# Round 3: k_emb_final's adjacency workgroup on the second stream beside k_emb_combine -- A/B via
# REDCLIFF_ADJ_FORK (interleaved), full GPU suite, D4IC / TST timelines
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
B="python bench.py --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0"
for cfg in d4ic c1k4 c4; do
  step zl_off_$cfg 200 env REDCLIFF_ADJ_FORK=0 $B --config $cfg
  step zl_on_$cfg 200 $B --config $cfg
done
step zl_off2_d4ic 200 env REDCLIFF_ADJ_FORK=0 $B --config d4ic
step zl_on2_d4ic 200 $B --config d4ic
step zl_trace_d4ic 200 python -u scripts/phase_trace.py --config d4ic
step zl_suite 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --durations=5
kill $HB
