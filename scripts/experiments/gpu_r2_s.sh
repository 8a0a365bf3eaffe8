#!/bin/bash
# GC-progress kernel (1024-thread workgroups, compacted ROC pairs, register-blocked powers):
# metric tests, kernel time at D4IC / C5 shapes, kernel trace of the C5 fit (validation cost)
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step r2_metrics 300 python -u -m pytest tests/test_gc_metrics.py tests/test_gpu_pack_fit.py -m gpu -x -v --timeout 240 --timeout-method thread
step r2_gck_c5 300 python -u scripts/pack_fit_profile.py --config c5 --replicas 2 --epochs 3 --train-batches 2 --gc-kernel
step r2_gck_d4ic 300 python -u scripts/pack_fit_profile.py --config d4ic --replicas 2 --epochs 3 --train-batches 2 --gc-kernel
step r2_c5_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5trace -o run -- python scripts/fit_profile.py --config c5 --train-batches 10 --epochs 3
kill $HB
