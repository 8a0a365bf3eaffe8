#!/bin/bash
# full GPU suite on the merged-backward build, bench (default + C1K4 check)
source "$(dirname "$0")/../gpu_steps.sh"
step r2_suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step r2_bench 600 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 5
step r2_c1k4 200 python -u bench.py --config c1k4 --steps 50 --warmup 10 --no-cpu-baseline --replicas 1 --fit-replicas 0 --no-north-star
