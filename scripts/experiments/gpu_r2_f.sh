#!/bin/bash
# Whole-fit profile (D4IC, C1K4): where an epoch's wall clock goes.
source "$(dirname "$0")/../gpu_steps.sh"
step r2_fitprof_d4ic 300 python -u scripts/fit_profile.py --config d4ic --epochs 20
step r2_fitprof_c1k4 300 python -u scripts/fit_profile.py --config c1k4 --epochs 20
step r2_trace_d4ic 200 python -u scripts/phase_trace.py --config d4ic
