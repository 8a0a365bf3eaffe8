#!/bin/bash
# merged vs two-launch backward at the C1(K=4) north-star config and C4
source "$(dirname "$0")/../gpu_steps.sh"
for cfg in c1k4 c4; do
step r2_${cfg}_merged 200 python -u bench.py --config $cfg --steps 50 --warmup 10 --no-cpu-baseline --replicas 1 --fit-replicas 0 --no-north-star
export REDCLIFF_MERGE=0; step r2_${cfg}_two 200 python -u bench.py --config $cfg --steps 50 --warmup 10 --no-cpu-baseline --replicas 1 --fit-replicas 0 --no-north-star; unset REDCLIFF_MERGE
done
