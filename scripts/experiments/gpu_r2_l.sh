#!/bin/bash
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step r2_merged 300 python -u -m pytest tests/test_gpu_forked.py tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py -v --timeout 240 --timeout-method thread
step r2_bench_m 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --fit-replicas 0 --replicas 1
S="python bench.py --no-cpu-baseline --no-kernel-times --steps 30 --warmup 3 --replicas 1 --fit-replicas 0 --no-north-star"
step r2_pmc_fetch_s 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_s -o run -- $S
step r2_pmc_write_s 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_s -o run -- $S
kill $HB
