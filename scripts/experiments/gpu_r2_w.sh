#!/bin/bash
# cached replica index tensors (no pageable H2D in the packed epoch): pack tests, pack profiles
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step r2_packtests 400 python -u -m pytest tests/test_gpu_pack_fit.py tests/test_gpu_replicas.py -m gpu -x -v --timeout 240 --timeout-method thread
step r2_packprof_d4ic 300 python -u scripts/pack_fit_profile.py --config d4ic --cprofile
kill $HB
