#!/bin/bash
# device tracker statistics (L1 / cosine) + cached truth: whole GPU suite, fit profiles
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step r2_suite 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
step r2_packprof_d4ic 300 python -u scripts/pack_fit_profile.py --config d4ic
step r2_packprof_c5 300 python -u scripts/pack_fit_profile.py --config c5 --replicas 4 --epochs 6 --train-batches 4
step r2_fitprof_d4ic 300 python -u scripts/fit_profile.py --config d4ic
step r2_fitprof_c5 300 python -u scripts/fit_profile.py --config c5 --train-batches 10
kill $HB
