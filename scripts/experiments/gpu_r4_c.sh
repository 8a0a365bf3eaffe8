#!/bin/bash
# Round 4: batched embedder v2 (tile workgroups) -- tests, grid A/B (factor-kernel LDS variants with the
# GEMM embedder; batched v2 vs GEMM embedder), kernel stats and LDS counters of the batched kernels.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step c_tests 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_replicas.py tests/test_gpu_parity.py -k "replicas or embbatched or C2"
G="python scripts/grid_step.py --replicas 128 --steps 30"
step c_grid_prev 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so $G
step c_grid_xsonly_gemm 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_xsonly.so REDCLIFF_EMB_PATH=gemm $G
step c_grid_cur_gemm 200 env REDCLIFF_EMB_PATH=gemm $G
step c_grid_cur 200 env REDCLIFF_EMB_PATH=batched $G
step c_grid_prev2 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so $G
step c_grid_xsonly_gemm2 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_xsonly.so REDCLIFF_EMB_PATH=gemm $G
step c_grid_cur_gemm2 200 env REDCLIFF_EMB_PATH=gemm $G
step c_grid_cur2 200 env REDCLIFF_EMB_PATH=batched $G
step c_stats 200 env REDCLIFF_EMB_PATH=batched rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d gpurun_out/stats_c -o run -- python scripts/grid_step.py --replicas 128 --steps 20
step c_lds 150 env REDCLIFF_EMB_PATH=batched rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-include-regex k_ --output-format csv -d gpurun_out/pmc_c_lds -o run -- python scripts/grid_step.py --replicas 128 --steps 3
step c_tests2 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pack_fit.py
step c_ns 200 python scripts/ns_probe.py
step c_ns_nccl 200 python scripts/ns_probe.py --nccl
kill $HB
