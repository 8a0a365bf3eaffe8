#!/bin/bash
# Round 3: TST-shaped single fit with the GEMM-shaped embedder / more windows per forward workgroup.
source "$(dirname "$0")/../gpu_steps.sh"
C="python bench.py --config c4 --steps 200 --warmup 20 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0 --no-kernel-times"
step u_default 300 $C
step u_gemm 300 env REDCLIFF_EMB_PATH=gemm $C
step u_sb2 300 env REDCLIFF_EMB_SB=2 $C
step u_sb4 300 env REDCLIFF_EMB_SB=4 $C
step u_gemm_stats 300 env REDCLIFF_EMB_PATH=gemm rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d gpurun_out/stats_u -o run -- $C
