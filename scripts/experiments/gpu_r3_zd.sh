#!/bin/bash
# Round 3: two-rank data-parallel tests with the fused update on / off
source "$(dirname "$0")/../gpu_steps.sh"
step zd_fused 300 python -u -m pytest tests/test_gpu_data_parallel.py -v --timeout 120 --timeout-method thread -k two_rank_data_parallel_matches
step zd_unfused 300 env REDCLIFF_DP_FUSED=0 python -u -m pytest tests/test_gpu_data_parallel.py -v --timeout 120 --timeout-method thread -k two_rank_data_parallel_matches
