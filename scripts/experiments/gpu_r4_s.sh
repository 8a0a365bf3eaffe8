#!/bin/bash
# Round 4: packed grid step (R=128 D4IC) under the tuning knobs; kernel stats of the grid step
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4s
step s_sweep 500 python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2
step s_grid_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4s/prof -o grid -- python3 scripts/grid_step.py --replicas 128 --steps 20
kill $HB
