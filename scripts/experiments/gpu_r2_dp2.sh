#!/bin/bash
# Round 2: the large-shard factor-path fallback test.
source "$(dirname "$0")/../gpu_steps.sh"
step dp2_tests 300 python -u -m pytest tests/test_gpu_data_parallel.py -x -v --timeout 200 --timeout-method thread
