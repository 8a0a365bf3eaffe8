#!/bin/bash
# Round 5: where the embedder backward's node staging (phase 33 -> 34, 7-10 us) spends its time: marks
# after the staging pass (44), the first dL/dw round (45), the remaining rounds (46); a timing-only
# trace build stages the window operands a second time (mark 47: warm caches / TLB).
source "$(dirname "$0")/../gpu_steps.sh"
for cfg in c1k4 c4; do
  step aj_trace_$cfg 200 python scripts/phase_trace.py --config $cfg
  REDCLIFF_TRACE_LIB=scripts/bin/lib_stage2.so step aj_trace2_$cfg 200 python scripts/phase_trace.py --config $cfg
done
