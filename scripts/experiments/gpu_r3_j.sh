#!/bin/bash
# Round 3: counter passes of the R = 128 grid step (factor s16 kernels, embedder chain) and the
# single-fit phase timeline of HEAD.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
G="python scripts/grid_step.py --replicas 128 --steps 3"
F="--kernel-include-regex k_ --output-format csv"
step j_g_sq1 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT $F -d gpurun_out/pmc_j_g_sq1 -o run -- $G
step j_g_sq2 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE $F -d gpurun_out/pmc_j_g_sq2 -o run -- $G
step j_g_fetch 150 rocprofv3 --pmc FETCH_SIZE $F -d gpurun_out/pmc_j_g_fetch -o run -- $G
step j_g_write 150 rocprofv3 --pmc WRITE_SIZE $F -d gpurun_out/pmc_j_g_write -o run -- $G
kill $HB
