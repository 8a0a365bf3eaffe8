#!/bin/bash
# Round 3: fused data-parallel update (redcliff_dp_update), default-priority aux stream, split-lead
# step for small update grids -- full GPU suite, DP bench at B=128, single-fit bench lines.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step ze_suite 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --durations=5
step ze_dpbench 300 python bench.py --mode dp --dp-batch 128 --steps 300 --warmup 30
step ze_dp_c4 200 python -u scripts/dp_profile.py --batch 128 --steps 200
step ze_c1k4 300 python bench.py --config c1k4 --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step ze_c4 300 python bench.py --config c4 --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step ze_c5 300 python bench.py --config c5 --steps 100 --warmup 10 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
kill $HB
