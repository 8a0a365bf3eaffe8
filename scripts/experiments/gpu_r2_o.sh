#!/bin/bash
# Whole-fit breakdown of the current build (D4IC, C5) and the R = 32 packed-grid PMC passes.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step r2_fitprof_d4ic 300 python -u scripts/fit_profile.py --config d4ic
step r2_fitprof_c5 300 python -u scripts/fit_profile.py --config c5 --train-batches 10
G="python bench.py --no-cpu-baseline --no-kernel-times --steps 3 --warmup 1 --replicas 32 --grid-steps 5 --fit-replicas 0 --no-north-star"
step r2_pmc_fetch_g 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_g -o run -- $G
step r2_pmc_write_g 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_g -o run -- $G
kill $HB
