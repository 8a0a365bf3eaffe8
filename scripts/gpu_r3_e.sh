#!/bin/bash
# Round 3: C5 gate / tail classification, the trimmed matrix-core k-loops across the suites that
# pin them (pack == single, autograd, fit modes), and the bench line with <= 15 CPU workers.
source "$(dirname "$0")/gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step e_c5 400 python -u -m pytest "tests/test_gpu_parity.py::test_stress_config_error_budget_vs_fp64" -v -s --timeout 360 --timeout-method thread
step e_tests 500 python -u -m pytest tests/test_gpu_autograd.py tests/test_gpu_fit_modes.py tests/test_gpu_status.py tests/test_gpu_forked.py tests/test_gpu_pack_fit.py -v --timeout 200 --timeout-method thread --durations=10
step e_bench 500 python -u bench.py --steps 200 --warmup 20
kill $HB
