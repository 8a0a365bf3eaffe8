#!/bin/bash
# Round 4: multi-rank --mode fit rehearsal on one GPU (2 ranks share cuda:0): gloo coordination,
# no RCCL communicator in the single-fit / grid / fits-per-hour legs; the one-rank default line
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step ad_two 600 python bench.py --gpus 2 --steps 20 --warmup 5 --replicas 16 --grid-steps 20 --fit-replicas 16 --fit-epochs 6 --dp-leg-batch 0 --no-cpu-baseline
step ad_one 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
kill $HB
