#!/bin/bash
# Round 6: per-workgroup trace of the R = 128 D4IC packed step (trace build), factor chain on one stream,
# with k_fac_mix's phase marks (workgroup 0 of replica 0).
source "$(dirname "$0")/../gpu_steps.sh"
REDCLIFF_FORK=0 step j_trace 300 python scripts/phase_trace_pack.py --replicas 128 --steps 6
REDCLIFF_FORK=0 step j_trace_c4 300 python scripts/phase_trace_pack.py --replicas 128 --steps 6 --config c4
