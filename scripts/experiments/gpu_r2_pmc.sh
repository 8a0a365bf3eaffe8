#!/bin/bash
# Round-2 PMC passes of the current build (FETCH / WRITE, one counter per run) over the single
# D4IC fit and over the R = 32 packed grid; bench.py reads them back (smallest grid = single
# fit, largest = the packed launches).  A heartbeat keeps the silent counter runs visible.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
S="python bench.py --no-cpu-baseline --no-kernel-times --steps 30 --warmup 3 --replicas 1 --fit-replicas 0 --no-north-star"
G="python bench.py --no-cpu-baseline --no-kernel-times --steps 3 --warmup 1 --replicas 32 --grid-steps 5 --fit-replicas 0 --no-north-star"
step r2_pmc_fetch_s 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_s -o run -- $S
step r2_pmc_write_s 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_s -o run -- $S
step r2_pmc_fetch_g 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_g -o run -- $G
step r2_pmc_write_g 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_g -o run -- $G
kill $HB
