#!/bin/bash
# Round 4: conflict-free LDS layouts in k_fac_fwd_s16 / k_fac_bwd_s16 (bitwise against the previous
# build, matrix-core factor path forced) and the replica-batched embedder kernels -- tests first,
# then grid timing A/B, LDS counter passes, kernel stats, the default bench line.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step b_tests 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_replicas.py tests/test_gpu_parity.py -k "replicas or embbatched or embgemm or C2"
export REDCLIFF_FAC_PATH=mfma
step b_dump_prev 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python scripts/compare_builds.py dump gpurun_out/prev.npz
step b_dump_cur 200 python scripts/compare_builds.py dump gpurun_out/cur.npz
step b_cmp 60 python scripts/compare_builds.py compare gpurun_out/prev.npz gpurun_out/cur.npz
unset REDCLIFF_FAC_PATH
step b_grid_prev 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python scripts/grid_step.py --replicas 128 --steps 30
step b_grid_cur_gemm 200 env REDCLIFF_EMB_PATH=gemm python scripts/grid_step.py --replicas 128 --steps 30
step b_grid_cur 200 python scripts/grid_step.py --replicas 128 --steps 30
step b_grid_prev2 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python scripts/grid_step.py --replicas 128 --steps 30
step b_grid_cur2 200 python scripts/grid_step.py --replicas 128 --steps 30
G="python scripts/grid_step.py --replicas 128 --steps 3"
F="--kernel-include-regex k_ --output-format csv"
step b_lds_cur 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES $F -d gpurun_out/pmc_b_lds_cur -o run -- $G
step b_lds_prev 150 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES $F -d gpurun_out/pmc_b_lds_prev -o run -- $G
step b_stats 200 rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d gpurun_out/stats_b -o run -- python scripts/grid_step.py --replicas 128 --steps 20
step b_tests2 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pack_fit.py tests/test_gpu_data_parallel.py tests/test_gpu_wavelet.py tests/test_gpu_fit_golden.py
step b_bench20 400 python bench.py --steps 20 --warmup 5
kill $HB
