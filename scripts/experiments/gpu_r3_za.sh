#!/bin/bash
# Round 3: second stream next to RCCL -- is the aux stream's priority the cause of the 3x slower
# forked step once a nccl process group exists?
source "$(dirname "$0")/../gpu_steps.sh"
step za_prio_normal 200 env REDCLIFF_SPLIT_LEAD=1 REDCLIFF_AUX_PRIO=normal python -u scripts/dp_profile.py --config c1k4 --batch 128 --steps 200
step za_prio_high 200 env REDCLIFF_SPLIT_LEAD=1 REDCLIFF_AUX_PRIO=high python -u scripts/dp_profile.py --config c1k4 --batch 128 --steps 200
step za_queues8 200 env REDCLIFF_SPLIT_LEAD=1 GPU_MAX_HW_QUEUES=8 python -u scripts/dp_profile.py --config c1k4 --batch 128 --steps 200
