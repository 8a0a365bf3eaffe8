#!/bin/bash
# grouped validation: bitwise test + the parity tests that validate, then the D4IC fit profile
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step r2_val 400 python -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_parity.py tests/test_gpu_pack_fit.py tests/test_gpu_checkpoint.py -m gpu -x -v --timeout 240 --timeout-method thread
step r2_fitprof_d4ic 300 python -u scripts/fit_profile.py --config d4ic
step r2_fitprof_c5 300 python -u scripts/fit_profile.py --config c5 --train-batches 10
kill $HB
