#!/bin/bash
# Round 2: new boundary / packed-fit / checkpoint tests, the whole GPU suite, a first bench line.
source "$(dirname "$0")/../gpu_steps.sh"
step r2_new_tests 600 python -u -m pytest tests/test_gpu_autograd.py tests/test_gpu_pack_fit.py tests/test_gpu_checkpoint.py -v --timeout 300 --timeout-method thread
step r2_gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step r2_bench 600 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 5
