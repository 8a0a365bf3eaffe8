#!/bin/bash
# Round 2: factor re-ordering ("pretrain_factor" modes) and Freeze* modes, then the fit tests
# that share the changed fit loop.
source "$(dirname "$0")/../gpu_steps.sh"
step r2_fit_modes 400 python -u -m pytest tests/test_gpu_fit_modes.py -x -v --timeout 200 --timeout-method thread
step r2_fit_related 600 python -u -m pytest tests/test_gpu_pack_fit.py tests/test_gpu_checkpoint.py -x -v --timeout 300 --timeout-method thread
