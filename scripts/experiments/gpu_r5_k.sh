#!/bin/bash
# Round 5: (1) GEMM-core replica axis fix (single-entry active lists): replica / pack-fit tests;
# (2) channel-sliced embedder forward (REDCLIFF_EMB_FWD_COLS) single-fit sweep at C1(K=4) / TST / D4IC
# against the previous build; (3) parity and pack tests with the sliced forward forced; phase trace
source "$(dirname "$0")/../gpu_steps.sh"
P=scripts/bin/lib_prev_r5k.so
T="python -u -m pytest -v --timeout 300 --timeout-method thread -rA"
step k_tests 900 $T tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
for cfg in c1k4 c4 d4ic; do
  REDCLIFF_HIP_LIB=$P step k_prev_${cfg}_$rep 200 $B --config $cfg
  for cols in 0 600 300 200 100; do
    REDCLIFF_EMB_FWD_COLS=$cols step k_cols_${cfg}_${cols}_$rep 200 $B --config $cfg
  done
done
done
REDCLIFF_EMB_FWD_COLS=200 step k_parity_split 900 $T tests/test_gpu_parity.py tests/test_gpu_fit_golden.py tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py tests/test_gpu_forked.py
REDCLIFF_EMB_FWD_COLS=200 step k_trace_c1k4 200 python scripts/phase_trace.py --config c1k4
step k_trace_c1k4_0 200 python scripts/phase_trace.py --config c1k4
