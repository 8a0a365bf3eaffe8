#!/bin/bash
# Round 3: counter passes of the R = 128 grid step on the rewritten short-contraction kernels.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
G="python scripts/grid_step.py --replicas 128 --steps 3"
F="--kernel-include-regex k_fac --output-format csv"
step l_sq1 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT $F -d gpurun_out/pmc_l_sq1 -o run -- $G
step l_sq2 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE $F -d gpurun_out/pmc_l_sq2 -o run -- $G
step l_sq3 150 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_LEVEL_WAVES SQ_ACCUM_PREV_HIRES $F -d gpurun_out/pmc_l_sq3 -o run -- $G
step l_fetch 150 rocprofv3 --pmc FETCH_SIZE $F -d gpurun_out/pmc_l_fetch -o run -- $G
step l_write 150 rocprofv3 --pmc WRITE_SIZE $F -d gpurun_out/pmc_l_write -o run -- $G
kill $HB
