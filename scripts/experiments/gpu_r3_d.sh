#!/bin/bash
# Round 3: C5 / resume fixes, GEMM embedder batched over replicas (bitwise test, grid timing
# fused vs gemm), the bench line with the data-parallel leg, counter list.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step d_tests 500 python -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_fit_golden.py tests/test_gpu_data_parallel.py "tests/test_gpu_parity.py::test_stress_config_error_budget_vs_fp64" "tests/test_gpu_parity.py::test_published_configs_three_phases_vs_oracle" -v -s --timeout 300 --timeout-method thread --durations=10
step d_grid_fused 200 env REDCLIFF_EMB_PATH=fused python -u scripts/grid_step.py --replicas 128 --steps 20
step d_grid_gemm 200 python -u scripts/grid_step.py --replicas 128 --steps 20
step d_kt_gemm 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_grid_gemm -o run -- python scripts/grid_step.py --replicas 128 --steps 20
step d_bench 500 python -u bench.py --steps 200 --warmup 20
rocprofv3 -L > gpurun_out/d_counters.txt 2>&1 || true
kill $HB
