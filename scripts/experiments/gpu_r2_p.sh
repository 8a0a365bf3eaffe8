#!/bin/bash
# Packed-fit (fits/hour) breakdown at D4IC and C5 + the GC-progress kernel alone; the R = 32
# grid PMC passes restricted to the library's own kernels (the unrestricted pass hit an AQL
# packet-format abort in the profiler while the pack was being built).
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step r2_packprof_d4ic 300 python -u scripts/pack_fit_profile.py --config d4ic --gc-kernel
step r2_packprof_c5 300 python -u scripts/pack_fit_profile.py --config c5 --replicas 4 --epochs 6 --train-batches 4 --gc-kernel
G="python bench.py --no-cpu-baseline --no-kernel-times --steps 3 --warmup 1 --replicas 32 --grid-steps 5 --fit-replicas 0 --no-north-star"
step r2_pmc_fetch_g 200 rocprofv3 --kernel-include-regex "k_" --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_g -o run -- $G
step r2_pmc_write_g 200 rocprofv3 --kernel-include-regex "k_" --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_g -o run -- $G
kill $HB
