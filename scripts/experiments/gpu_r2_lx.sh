#!/bin/bash
# Round 2: k_emb_bwd with the window tile staged late into dead LDS (RC_EMB_LATE_X) and with
# waves-per-EU floors 5 / 6 -- grid R = 128 and single fit, plus the bitwise pack tests and the
# parity suite on the late-staging library.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
G="python -u bench.py --steps 50 --warmup 5 --fit-replicas 0 --no-cpu-baseline --no-north-star"
step lx_base 300 $G
for v in lx lx5 lx6; do
  REDCLIFF_HIP_LIB=$PWD/scripts/bin/lib_$v.so step lx_$v 300 $G
done
REDCLIFF_HIP_LIB=$PWD/scripts/bin/lib_lx.so step lx_tests 600 python -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py tests/test_gpu_parity.py tests/test_gpu_forked.py -x -v --timeout 300 --timeout-method thread
kill $HB
