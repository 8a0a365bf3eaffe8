#!/bin/bash
# Round 2: GEMM tile choice at C5 with the matrix-core core (default rule / 64 / 32).
source "$(dirname "$0")/../gpu_steps.sh"
C5="python -u bench.py --config c5 --steps 30 --warmup 5 --replicas 1 --fit-replicas 0 --no-cpu-baseline --no-north-star --no-kernel-times"
step tile_auto 300 $C5
REDCLIFF_GEMM_TILE=64 step tile_64 300 $C5
REDCLIFF_GEMM_TILE=32 step tile_32 300 $C5
step tile_auto2 300 $C5
