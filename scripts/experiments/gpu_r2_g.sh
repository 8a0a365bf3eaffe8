#!/bin/bash
# C5 fp32-realisation test, whole-fit profiles, D4IC workgroup trace.
source "$(dirname "$0")/../gpu_steps.sh"
step r2_c5 600 python -u -m pytest tests/test_gpu_parity.py -v -s -k stress --timeout 500 --timeout-method thread
# step r2_fitprof_d4ic 300 python -u scripts/fit_profile.py --config d4ic --epochs 20
# step r2_fitprof_c1k4 300 python -u scripts/fit_profile.py --config c1k4 --epochs 20
# step r2_trace_d4ic 200 python -u scripts/phase_trace.py --config d4ic
