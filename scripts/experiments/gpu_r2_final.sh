#!/bin/bash
# R = 128 grid PMC passes + kernel stats, then the driver's bench command
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
G="python bench.py --no-cpu-baseline --no-kernel-times --steps 3 --warmup 1 --replicas 128 --grid-steps 5 --fit-replicas 0 --no-north-star"
step r2_pmc_fetch_g 200 rocprofv3 --kernel-include-regex "k_" --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_g -o run -- $G
step r2_pmc_write_g 200 rocprofv3 --kernel-include-regex "k_" --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_g -o run -- $G
step r2_kstats_g 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kstats_g -o run -- $G
kill $HB
