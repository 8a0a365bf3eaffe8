#!/bin/bash
# Round 4: fit-level parity against the reference's own fits (envelope criterion), fit-mode and
# checkpoint suites, with the current build
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step h_fit 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_fit_golden.py
step h_suite 700 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_checkpoint.py tests/test_gpu_fit_modes.py tests/test_gpu_data_parallel.py tests/test_gpu_forked.py tests/test_gpu_status.py tests/test_gpu_wavelet.py
kill $HB
