#!/bin/bash
# Round 3: D4IC timeline after the matrix-core factor backward
source "$(dirname "$0")/../gpu_steps.sh"
step zr_trace_d4ic 200 python -u scripts/phase_trace.py --config d4ic
step zr_trace_c1k4 200 python -u scripts/phase_trace.py --config c1k4
