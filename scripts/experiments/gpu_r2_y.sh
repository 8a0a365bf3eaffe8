#!/bin/bash
# XCD-aware factor workgroup order in k_bwd_merged: bitwise tests, bench (HBM roofline, CPU
# fits/hour), PMC passes of the single fit
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step r2_merged 400 python -u -m pytest tests/test_gpu_forked.py tests/test_gpu_replicas.py tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread
step r2_bench 400 python -u bench.py --steps 20 --warmup 5
S="python bench.py --no-cpu-baseline --no-kernel-times --steps 30 --warmup 3 --replicas 1 --fit-replicas 0 --no-north-star"
step r2_pmc_fetch_s 240 rocprofv3 --kernel-include-regex "k_" --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_s -o run -- $S
step r2_pmc_write_s 240 rocprofv3 --kernel-include-regex "k_" --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_s -o run -- $S
kill $HB
