#!/bin/bash
# Round 2: the fp32 matrix-core GEMM core (rc_gemm.h k_rc_gemm_mfma) -- the tests that run the
# GEMM-shaped embedder and the generic path, then C5 with each core and the kernel stats.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step r2_gemm_tests 600 python -u -m pytest tests/test_gpu_generic.py tests/test_gpu_parity.py tests/test_gpu_fit_modes.py -v --timeout 300 --timeout-method thread
C5="python -u bench.py --config c5 --steps 20 --warmup 5 --replicas 1 --fit-replicas 0 --no-cpu-baseline --no-north-star"
step r2_c5_mfma 300 $C5
REDCLIFF_GEMM_CORE=valu step r2_c5_valu 300 $C5
step r2_c5_kstats 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kstats_c5 -o run -- $C5
kill $HB
