#!/bin/bash
# Round 5: GPU suite on ABI 9 (mixed-schedule / per-replica packs, R = 128 pack, TST fit fixture + envelope,
# DP vs fixture), then the reference-grid fits/hour leg alone
source "$(dirname "$0")/../gpu_steps.sh"
step r5c_suite 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=12 -rA
step r5c_refgrid 600 python bench.py --steps 5 --warmup 2 --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --no-cpu-baseline --no-north-star --no-kernel-times
