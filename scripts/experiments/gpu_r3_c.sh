#!/bin/bash
# Round 3: fixed tests + merged-backward lead split (trace, bench).
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step c_tests 500 python -u -m pytest tests/test_gpu_fit_golden.py tests/test_gpu_status.py tests/test_gpu_autograd.py tests/test_gpu_fit_modes.py tests/test_gpu_forked.py "tests/test_gpu_parity.py::test_stress_config_error_budget_vs_fp64" -v -s --timeout 300 --timeout-method thread --durations=10
step c_trace 120 python -u scripts/phase_trace.py --config d4ic
step c_bench 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --fit-replicas 0 --dp-leg-batch 1024
kill $HB
