#!/bin/bash
# Round 2: fp64 error-budget stress test, configs[0] K=2, packed-fit bitwise test.
source "$(dirname "$0")/../gpu_steps.sh"
step r2_parity 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pack_fit.py -v -k "C1 or stress or pack_fit" --timeout 600 --timeout-method thread
