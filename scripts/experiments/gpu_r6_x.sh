#!/bin/bash
# Round 6: the lag-64 fit fixture's GPU tests with the float64 realization in its envelope, and the
# GPU fit against the reference's own float64 fit.
source "$(dirname "$0")/../gpu_steps.sh"
step x_lag64 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_fit_golden.py -k "lag64"
