#!/bin/bash
# Round 4: merged backward forced at C1(K=4) / TST (grid not resident) vs the default split-lead step
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
for i in 1 2; do
step as_def$i 200 python -u scripts/ab_single.py --tag default --configs c1k4,c4
step as_merge$i 200 env REDCLIFF_MERGE=1 python -u scripts/ab_single.py --tag merge1 --configs c1k4,c4
step as_nosplit$i 200 env REDCLIFF_SPLIT_LEAD=0 python -u scripts/ab_single.py --tag nosplit --configs c1k4,c4
done
kill $HB
