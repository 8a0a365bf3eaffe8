#!/bin/bash
# Round 3: rewritten short-contraction factor kernels -- bitwise against the previous build
# (matrix-core path forced), the factor-path GPU tests, R = 128 grid timing old vs new, kernel stats.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
export REDCLIFF_FAC_PATH=mfma
step k_dump_prev 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python scripts/compare_builds.py dump gpurun_out/prev.npz
step k_dump_cur 200 python scripts/compare_builds.py dump gpurun_out/cur.npz
step k_cmp 60 python scripts/compare_builds.py compare gpurun_out/prev.npz gpurun_out/cur.npz
unset REDCLIFF_FAC_PATH
step k_tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py tests/test_gpu_parity.py tests/test_gpu_forked.py tests/test_gpu_fit_modes.py tests/test_gpu_data_parallel.py
step k_grid_prev 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python scripts/grid_step.py --replicas 128 --steps 30
step k_grid_cur 200 python scripts/grid_step.py --replicas 128 --steps 30
step k_stats 200 rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d gpurun_out/stats_k -o run -- python scripts/grid_step.py --replicas 128 --steps 20
kill $HB
