#!/bin/bash
# Round 3: counter list, then SQ / TCC counter passes (own kernels only) of the R = 128 grid step
# and of the single-fit bench leg.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step h_list 60 rocprofv3 -L
G="python scripts/grid_step.py --replicas 128 --steps 3"
S="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-north-star --no-kernel-times --replicas 1 --fit-replicas 0 --dp-leg-batch 0"
F="--kernel-include-regex ^k_ --output-format csv"
step h_g_sq1 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT $F -d gpurun_out/pmc_h_g_sq1 -o run -- $G
step h_s_sq1 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT $F -d gpurun_out/pmc_h_s_sq1 -o run -- $S
step h_g_fetch 150 rocprofv3 --pmc FETCH_SIZE $F -d gpurun_out/pmc_h_g_fetch -o run -- $G
step h_g_write 150 rocprofv3 --pmc WRITE_SIZE $F -d gpurun_out/pmc_h_g_write -o run -- $G
kill $HB
