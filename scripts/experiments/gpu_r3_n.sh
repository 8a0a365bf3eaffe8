#!/bin/bash
# Round 3: one combined step on the matrix-core factor path, round-start build vs current, per tensor.
source "$(dirname "$0")/../gpu_steps.sh"
export COMPARE_EPOCHS=2 COMPARE_ONE_BATCH=1 COMPARE_SHOW=30
step n_dump_prev 200 env REDCLIFF_FAC_PATH=mfma REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python scripts/compare_builds.py dump gpurun_out/prev1.npz
step n_dump_cur 200 env REDCLIFF_FAC_PATH=mfma python scripts/compare_builds.py dump gpurun_out/cur1.npz
step n_cmp 60 python scripts/compare_builds.py compare gpurun_out/prev1.npz gpurun_out/cur1.npz
step n_tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py tests/test_gpu_parity.py tests/test_gpu_forked.py tests/test_gpu_fit_modes.py tests/test_gpu_data_parallel.py
step n_grid_cur 200 python scripts/grid_step.py --replicas 128 --steps 30
step n_stats 200 rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d gpurun_out/stats_n -o run -- python scripts/grid_step.py --replicas 128 --steps 20
