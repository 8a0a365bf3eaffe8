#!/bin/bash
# merged backward: bitwise test first, then the GPU suite and the bench.
source "$(dirname "$0")/../gpu_steps.sh"
step r2_merged 300 python -u -m pytest tests/test_gpu_forked.py tests/test_gpu_replicas.py -v --timeout 240 --timeout-method thread
step r2_bench_m 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 2 --fit-replicas 0
