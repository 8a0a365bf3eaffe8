#!/bin/bash
# Round 3: counters of the R = 128 grid step (factor kernels on the matrix cores, embedder chain)
# and the single-fit phase timeline with the factor leads' publish times.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
G="python scripts/grid_step.py --replicas 128 --steps 3"
step g_trace 200 python -u scripts/phase_trace.py --config d4ic
step g_pmc_sq1 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc_g_sq1 -o run -- $G
step g_pmc_sq2 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_g_sq2 -o run -- $G
step g_pmc_fetch 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_g_fetch -o run -- $G
step g_pmc_write 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_g_write -o run -- $G
kill $HB
