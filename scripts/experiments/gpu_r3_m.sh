#!/bin/bash
# Round 3: short-contraction factor kernels v3 (lane-linear buffer loads, LDS tiles) -- factor-path
# GPU tests, R = 128 grid timing against the round's starting build, kernel stats.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step m_tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py tests/test_gpu_parity.py tests/test_gpu_forked.py tests/test_gpu_fit_modes.py tests/test_gpu_data_parallel.py
step m_grid_prev 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python scripts/grid_step.py --replicas 128 --steps 30
step m_grid_cur 200 python scripts/grid_step.py --replicas 128 --steps 30
step m_stats 200 rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d gpurun_out/stats_m -o run -- python scripts/grid_step.py --replicas 128 --steps 20
kill $HB
