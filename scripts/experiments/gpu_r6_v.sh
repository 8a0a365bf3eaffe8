#!/bin/bash
# Round 6: drift of the GPU fit from the reference's lag-64 / 3-layer TST fit (fit_tst_lag64) on three
# kernel paths with different rounding orders (single-fit default, fc1 in 100-column slices, the packed
# grid's matrix-core factor + GEMM-shaped embedder kernels), and fit_tst for comparison.
source "$(dirname "$0")/../gpu_steps.sh"
step v_lag64_default 300 python tests/diagnostics/fit_drift.py fit_tst_lag64
REDCLIFF_EMB_FWD_COLS=100 step v_lag64_cols100 300 python tests/diagnostics/fit_drift.py fit_tst_lag64
REDCLIFF_FAC_PATH=mfma REDCLIFF_EMB_PATH=gemm step v_lag64_packed 300 python tests/diagnostics/fit_drift.py fit_tst_lag64
step v_tst_default 300 python tests/diagnostics/fit_drift.py fit_tst
REDCLIFF_FAC_PATH=mfma REDCLIFF_EMB_PATH=gemm step v_tst_packed 300 python tests/diagnostics/fit_drift.py fit_tst
