#!/bin/bash
# Round 4: where a packed fit's epoch goes on the device (kernel stats of ReplicaPack.fit), the
# default bench line with the RCCL group created for the data-parallel leg only, the DP leg alone.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step d_packfit 300 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --train-batches 8
step d_packfit_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_d -o run -- python scripts/pack_fit_profile.py --replicas 128 --epochs 40 --train-batches 8
step d_bench 500 python bench.py --steps 20 --warmup 5
step d_dp 300 python bench.py --mode dp --dp-batch 128 --steps 200 --warmup 20
kill $HB
