#!/bin/bash
# Round 6: the grid shape classes against the oracle (TST embed_lag x layers, synthetic K / p extremes,
# single-fit and packed kernels), the new K = 1 / K = 10 golden scenarios, the 256-replica TST pack.
source "$(dirname "$0")/../gpu_steps.sh"
step a_parity 900 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -rA \
  -k "grid_shape_classes or k1p3 or k10p6" --durations=10
step a_pack256 600 python -u -m pytest tests/test_gpu_large_pack.py -v --timeout 500 --timeout-method thread -rA \
  -k "256" --durations=5
step a_dp_generic 600 python -u -m pytest tests/test_gpu_data_parallel.py tests/test_gpu_generic.py tests/test_gpu_fit_golden.py -v \
  --timeout 300 --timeout-method thread -rA -k "data_parallel or sharded or fit_matches or hip_adam or two_rank" --durations=5
