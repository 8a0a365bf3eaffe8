#!/bin/bash
# Round 4: batched embedder v3 (LDS-staged operands, dS on the matrix cores, chunked head gradients):
# parity / replica tests on the path, grid A/B against the GEMM chain, kernel stats.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step e_tests 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_replicas.py tests/test_gpu_parity.py -k "replicas or embbatched"
G="python scripts/grid_step.py --replicas 128 --steps 30"
step e_grid_gemm 200 env REDCLIFF_EMB_PATH=gemm $G
step e_grid_batched 200 env REDCLIFF_EMB_PATH=batched $G
step e_grid_gemm2 200 env REDCLIFF_EMB_PATH=gemm $G
step e_grid_batched2 200 env REDCLIFF_EMB_PATH=batched $G
step e_stats 200 env REDCLIFF_EMB_PATH=batched rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d gpurun_out/stats_e -o run -- python scripts/grid_step.py --replicas 128 --steps 20
kill $HB
