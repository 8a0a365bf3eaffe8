#!/bin/bash
# Round 5: where the D4IC step (the bench `value`: forward, merged backward, embedder tail) spends its
# time after the latency work: phase traces.
source "$(dirname "$0")/../gpu_steps.sh"
step ap_trace_d4ic 200 python scripts/phase_trace.py --config d4ic
step ap_trace_d4ic2 200 python scripts/phase_trace.py --config d4ic
