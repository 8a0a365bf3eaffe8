#!/bin/bash
# Round 3: fused data-parallel update against the per-group Adam sequence; default-priority aux
# stream next to RCCL (split-lead C1(K=4) step inside a nccl process group)
source "$(dirname "$0")/../gpu_steps.sh"
step zc_tests 300 python -u -m pytest tests/test_gpu_data_parallel.py tests/test_gpu_forked.py -v --timeout 120 --timeout-method thread
step zc_dp_c1k4 200 python -u scripts/dp_profile.py --config c1k4 --batch 128 --steps 200
step zc_dp_c4 200 python -u scripts/dp_profile.py --batch 128 --steps 200
