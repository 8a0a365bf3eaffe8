#!/bin/bash
# Round 3: split-lead step gated on the update grid; is a second stream slow next to RCCL?
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step z_dp_c4 200 python -u scripts/dp_profile.py --batch 128 --steps 200
step z_dp_c1k4_s0 200 env REDCLIFF_SPLIT_LEAD=0 python -u scripts/dp_profile.py --config c1k4 --batch 128 --steps 200
step z_dp_c1k4_s1 200 env REDCLIFF_SPLIT_LEAD=1 python -u scripts/dp_profile.py --config c1k4 --batch 128 --steps 200
step z_c4 300 python bench.py --config c4 --steps 200 --warmup 20 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step z_c1k4 300 python bench.py --config c1k4 --steps 200 --warmup 20 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step z_fork 300 python -u -m pytest tests/test_gpu_forked.py tests/test_gpu_data_parallel.py -v --timeout 120 --timeout-method thread
kill $HB
