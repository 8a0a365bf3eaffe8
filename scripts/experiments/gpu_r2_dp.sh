#!/bin/bash
# Round 2: the data-parallel leg (configs[3] TST-shaped DataParallelFit) on one rank over RCCL,
# global batch 128 and 512 (512 windows per rank: the vector factor backward's LDS budget is
# exceeded there, so the matrix-core factor path takes over), then the DP GPU tests.
source "$(dirname "$0")/../gpu_steps.sh"
step dp_b128 300 python -u bench.py --mode dp --steps 50 --warmup 5 --no-cpu-baseline
step dp_b512 300 python -u bench.py --mode dp --steps 50 --warmup 5 --no-cpu-baseline --dp-batch 512
step dp_tests 300 python -u -m pytest tests/test_gpu_data_parallel.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread
