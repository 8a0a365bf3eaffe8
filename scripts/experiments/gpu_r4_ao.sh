#!/bin/bash
# Round 4: single-fit HBM passes (D4IC) on the network-major y build
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4ao
S="python bench.py --steps 30 --warmup 5 --preheat-s 0 --no-cpu-baseline --no-north-star --no-kernel-times --replicas 1 --fit-replicas 0 --dp-leg-batch 0"
F="--kernel-include-regex k_ --output-format csv"
step ao_fetch 150 rocprofv3 --pmc FETCH_SIZE $F -d gpurun_out/r4ao/pmc_s_fetch -o run -- $S
step ao_write 150 rocprofv3 --pmc WRITE_SIZE $F -d gpurun_out/r4ao/pmc_s_write -o run -- $S
kill $HB
