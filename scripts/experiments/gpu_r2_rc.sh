#!/bin/bash
# MFMA backward recomputes activations + output-layer grads (p*L <= 64): bitwise vs the previous
# build on the matrix-core path, then grid timing of prev / new (2 waves) / new (3 waves, spills)
source "$(dirname "$0")/../gpu_steps.sh"
export REDCLIFF_FAC_PATH=mfma
REDCLIFF_HIP_LIB=exp/lib_prev.so step rc_dump_prev 200 python -u scripts/compare_builds.py dump gpurun_out/prev.npz
step rc_dump_cur 200 python -u scripts/compare_builds.py dump gpurun_out/cur.npz
step rc_compare 100 python -u scripts/compare_builds.py compare gpurun_out/prev.npz gpurun_out/cur.npz
rm -f gpurun_out/prev.npz gpurun_out/cur.npz
unset REDCLIFF_FAC_PATH
G="python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-north-star --fit-replicas 0 --grid-steps 50 --replicas 32"
for v in prev cur prev cur; do
  if [ $v = cur ]; then step g_$v 200 $G; else REDCLIFF_HIP_LIB=exp/lib_$v.so step g_$v 200 $G; fi
  grep '^{' gpurun_out/g_$v.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); g=d['grid_search']; print('$v', g['windows_per_s'], g['ms_per_step'], g['roofline']['kernel_avg_us'])"
done
