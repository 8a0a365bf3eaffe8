#!/bin/bash
# Round 3: fused data-parallel update (redcliff_dp_update) -- DP tests, --mode dp bench at B=128,
# DP update profile; aux-stream priority low vs normal for the forked single fits (C1(K=4) split,
# C5 matrix-core fork).
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step zb_tests 300 python -u -m pytest tests/test_gpu_data_parallel.py tests/test_gpu_forked.py -v --timeout 120 --timeout-method thread
step zb_dpbench 300 python bench.py --mode dp --dp-batch 128 --steps 300 --warmup 30
step zb_dp 200 python -u scripts/dp_profile.py --batch 128 --steps 200
step zb_dpprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/zb_dpprof -o dp -- python -u scripts/dp_profile.py --batch 128 --steps 200
step zb_c1k4_low 300 env REDCLIFF_AUX_PRIO=low python bench.py --config c1k4 --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step zb_c1k4_norm 300 env REDCLIFF_AUX_PRIO=normal python bench.py --config c1k4 --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step zb_c5_low 300 env REDCLIFF_AUX_PRIO=low python bench.py --config c5 --steps 100 --warmup 10 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step zb_c5_norm 300 env REDCLIFF_AUX_PRIO=normal python bench.py --config c5 --steps 100 --warmup 10 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
kill $HB
