#!/bin/bash
# Round 3: R = 128 grid with the fused embedder (matrix-core node products) against the GEMM-shaped
# embedder, kernel stats of both.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step r_grid_gemm 200 python scripts/grid_step.py --replicas 128 --steps 30
step r_grid_fused 200 env REDCLIFF_EMB_PATH=fused python scripts/grid_step.py --replicas 128 --steps 30
step r_stats_fused 200 env REDCLIFF_EMB_PATH=fused rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d gpurun_out/stats_r_fused -o run -- python scripts/grid_step.py --replicas 128 --steps 20
step r_grid_gemm2 200 python scripts/grid_step.py --replicas 128 --steps 30
step r_grid_fused2 200 env REDCLIFF_EMB_PATH=fused python scripts/grid_step.py --replicas 128 --steps 30
kill $HB
