#!/bin/bash
# Round 2: late window staging + waves floor on the single-sub-block k_emb_bwd only (the merged
# single-fit kernel untouched): grid R = 128, single fit, north-star config; then the bitwise
# suites on the variant.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
G="python -u bench.py --steps 50 --warmup 5 --fit-replicas 0 --no-cpu-baseline"
step lx2_base 300 $G
for v in lx5b lx6b; do
  REDCLIFF_HIP_LIB=$PWD/scripts/bin/lib_$v.so step lx2_$v 300 $G
done
step lx2_base2 300 $G
REDCLIFF_HIP_LIB=$PWD/scripts/bin/lib_lx5b.so step lx2_tests 600 python -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py tests/test_gpu_parity.py tests/test_gpu_forked.py tests/test_gpu_fit_modes.py -x -v --timeout 300 --timeout-method thread
kill $HB
