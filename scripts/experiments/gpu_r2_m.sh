#!/bin/bash
# recomputed activations: bitwise equal to the previous build; then bench + PMC of the new build
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
export REDCLIFF_HIP_LIB=exp/lib_prev.so
step r2_dump_prev 200 python -u scripts/compare_builds.py dump gpurun_out/prev.npz
unset REDCLIFF_HIP_LIB
step r2_dump_cur 200 python -u scripts/compare_builds.py dump gpurun_out/cur.npz
step r2_compare 100 python -u scripts/compare_builds.py compare gpurun_out/prev.npz gpurun_out/cur.npz
rm -f gpurun_out/prev.npz gpurun_out/cur.npz
step r2_bench_m 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --fit-replicas 0 --replicas 1
S="python bench.py --no-cpu-baseline --no-kernel-times --steps 30 --warmup 3 --replicas 1 --fit-replicas 0 --no-north-star"
step r2_c1k4 200 python -u bench.py --config c1k4 --steps 50 --warmup 10 --no-cpu-baseline --replicas 1 --fit-replicas 0 --no-north-star
step r2_pmc_fetch_s 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_s -o run -- $S
step r2_pmc_write_s 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_s -o run -- $S
kill $HB
