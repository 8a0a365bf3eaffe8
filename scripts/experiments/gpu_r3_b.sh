#!/bin/bash
# Round 3: new parity tests (reference fit fixtures, reference-style resume, C5 two batches per
# phase with the fp32-oracle graph check, device status, data-parallel fit), then the whole GPU
# suite, a workgroup trace of the D4IC single-fit step and the data-parallel step breakdown.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
{ nproc; python -c "import os; print(os.cpu_count(), len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>&1; free -g; } > gpurun_out/b_host.txt 2>&1
step b_new 500 python -u -m pytest tests/test_gpu_fit_golden.py tests/test_gpu_status.py tests/test_gpu_checkpoint.py tests/test_gpu_data_parallel.py "tests/test_gpu_parity.py::test_stress_config_error_budget_vs_fp64" -v -s --timeout 300 --timeout-method thread --durations=12
step b_dpprof 180 python -u scripts/dp_profile.py --batch 128 --steps 200
step b_trace 120 python -u scripts/phase_trace.py --config d4ic
step b_suite 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=15
kill $HB
