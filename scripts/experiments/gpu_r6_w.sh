#!/bin/bash
# Round 6: where the GPU fit of fit_tst_lag64 leaves the reference (the oracle reproduces the
# reference's first epochs bit for bit on the CPU): per-tensor deviation from the oracle after each of
# the first training steps, the lag-64 fixture and fit_tst for comparison, single-fit and packed paths.
source "$(dirname "$0")/../gpu_steps.sh"
step w_lag64 300 python tests/diagnostics/step_drift.py fit_tst_lag64 4
REDCLIFF_FAC_PATH=mfma REDCLIFF_EMB_PATH=gemm step w_lag64_packed 300 python tests/diagnostics/step_drift.py fit_tst_lag64 2
step w_tst 300 python tests/diagnostics/step_drift.py fit_tst 4
