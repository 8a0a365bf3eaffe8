#!/bin/bash
# Round 3: C5 gate / tail classification; windowed small-node embedder kernels (pack == single,
# published-config parity on both product forms); trimmed matrix-core k-loops across the suites
# that pin them; grid timing + kernel trace; the bench line with <= 15 CPU workers.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step e_c5 400 python -u -m pytest "tests/test_gpu_parity.py::test_stress_config_error_budget_vs_fp64" -v -s --timeout 360 --timeout-method thread
step e_tests 600 python -u -m pytest tests/test_gpu_replicas.py "tests/test_gpu_parity.py::test_published_configs_three_phases_vs_oracle" tests/test_gpu_autograd.py tests/test_gpu_fit_modes.py tests/test_gpu_status.py tests/test_gpu_forked.py tests/test_gpu_pack_fit.py -v --timeout 200 --timeout-method thread --durations=10
step e_grid_tile 200 env REDCLIFF_FAC_FWD=tile REDCLIFF_FAC_BWD=tile REDCLIFF_EMB_WIN=0 python -u scripts/grid_step.py --replicas 128 --steps 20
step e_grid 200 python -u scripts/grid_step.py --replicas 128 --steps 20
step e_kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_grid_e -o run -- python scripts/grid_step.py --replicas 128 --steps 20
step e_bench 500 python -u bench.py --steps 200 --warmup 20
kill $HB
