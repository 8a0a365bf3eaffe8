#!/bin/bash
# Round 5: is the adjacency workgroup's chain in k_emb_final bound by instruction fetch?  Timing-only
# trace build (-DRC_ADJ_TWICE, wrong results) runs the normalize-A backward products and the supports
# twice in a row; marks 55 / 56 and 57 / 58 time each pass.
source "$(dirname "$0")/../gpu_steps.sh"
for cfg in c1k4 c4; do
  REDCLIFF_TRACE_LIB=scripts/bin/lib_adj2.so step ag_trace2_$cfg 200 python scripts/phase_trace.py --config $cfg
  step ag_trace_$cfg 200 python scripts/phase_trace.py --config $cfg
done
