#!/bin/bash
# Round 3: short-contraction kernels v4 (block operands one block ahead, two recompute chains per
# pass) and k_fac_mix slot sums loaded together -- factor-path tests, grid timing, counters, bpw sweep.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
G="python scripts/grid_step.py --replicas 128 --steps 3"
F="--kernel-include-regex k_fac --output-format csv"
step p_tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py tests/test_gpu_forked.py tests/test_gpu_fit_modes.py tests/test_gpu_data_parallel.py tests/test_gpu_wavelet.py
step p_grid 200 python scripts/grid_step.py --replicas 128 --steps 30
step p_stats 200 rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d gpurun_out/stats_p -o run -- python scripts/grid_step.py --replicas 128 --steps 20
step p_sq1 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT $F -d gpurun_out/pmc_p_sq1 -o run -- $G
step p_sq2 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE $F -d gpurun_out/pmc_p_sq2 -o run -- $G
for b in 4 8 16; do
  step p_bpw$b 200 env REDCLIFF_FAC_BPW=$b rocprofv3 --kernel-trace --stats --kernel-include-regex k_fac --output-format csv -d gpurun_out/stats_p_bpw$b -o run -- python scripts/grid_step.py --replicas 128 --steps 10
done
kill $HB
