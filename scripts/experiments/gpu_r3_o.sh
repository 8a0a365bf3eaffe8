#!/bin/bash
# Round 3: counters of the v3 short-contraction kernels (R = 128 grid) and a blocks-per-wave sweep.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
G="python scripts/grid_step.py --replicas 128 --steps 3"
F="--kernel-include-regex k_fac --output-format csv"
step o_sq1 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT $F -d gpurun_out/pmc_o_sq1 -o run -- $G
step o_sq2 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE $F -d gpurun_out/pmc_o_sq2 -o run -- $G
step o_fetch 150 rocprofv3 --pmc FETCH_SIZE $F -d gpurun_out/pmc_o_fetch -o run -- $G
step o_write 150 rocprofv3 --pmc WRITE_SIZE $F -d gpurun_out/pmc_o_write -o run -- $G
for b in 2 4 8 16; do
  step o_bpw$b 200 env REDCLIFF_FAC_BPW=$b rocprofv3 --kernel-trace --stats --kernel-include-regex k_fac --output-format csv -d gpurun_out/stats_o_bpw$b -o run -- python scripts/grid_step.py --replicas 128 --steps 10
done
kill $HB
