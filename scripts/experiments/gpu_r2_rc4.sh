#!/bin/bash
# recompute build: 4-epoch bitwise comparison vs the previous build (matrix-core path, forked
# single fits), the GPU suite, grid timing
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
export REDCLIFF_FAC_PATH=mfma
REDCLIFF_HIP_LIB=exp/lib_prev.so step rc_dump_prev 200 python -u scripts/compare_builds.py dump gpurun_out/prev.npz
step rc_dump_cur 200 python -u scripts/compare_builds.py dump gpurun_out/cur.npz
step rc_compare 100 python -u scripts/compare_builds.py compare gpurun_out/prev.npz gpurun_out/cur.npz
rm -f gpurun_out/prev.npz gpurun_out/cur.npz
unset REDCLIFF_FAC_PATH
step r2_suite 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
G="python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-north-star --fit-replicas 0 --grid-steps 50 --replicas 32"
step g_cur 200 $G
grep '^{' gpurun_out/g_cur.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); g=d['grid_search']; print('cur grid', g['windows_per_s'], g['ms_per_step'], g['roofline']['kernel_avg_us'])"
kill $HB
