#!/bin/bash
# C5 fp64 error-budget diagnostics (dumps the small tensors of HIP / oracle fp32 / oracle fp64).
source "$(dirname "$0")/../gpu_steps.sh"
export REDCLIFF_C5_DUMP=gpurun_out/c5_budget.npz
step r2_c5 1000 python -u -m pytest tests/test_gpu_parity.py -v -k stress --timeout 900 --timeout-method thread
