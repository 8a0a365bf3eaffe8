#!/bin/bash
# Round 6: workgroup / phase trace of the R = 128 TST pack step (k_fac_mix phases at K = 9).
source "$(dirname "$0")/../gpu_steps.sh"
REDCLIFF_FORK=0 step ee_trace_tst 300 python scripts/phase_trace_pack.py --replicas 128 --steps 6 --config c4
