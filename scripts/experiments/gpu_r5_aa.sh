#!/bin/bash
# Round 5: data-parallel fit with only the rank's shards resident (DataParallelFit.cache_dataset):
# bitwise against the whole-set layout, the fixture test of the 2-rank fit, the bench's DP leg
source "$(dirname "$0")/../gpu_steps.sh"
step aa_tests 900 python -u -m pytest tests/test_gpu_data_parallel.py tests/test_gpu_fit_golden.py -k "data_parallel or sharded or two_rank" -v --timeout 300 --timeout-method thread -rA
step aa_dp 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --ref-grid-epochs 0 --no-kernel-times
