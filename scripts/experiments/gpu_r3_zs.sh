#!/bin/bash
# Round 3: merged backward: factor leads split into record and update workgroups
# (same fmaf chains) -- bitwise comparison against the committed build, A/B interleaved, suite
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step zs_dump_prev 300 env REDCLIFF_HIP_LIB=scripts/bin/lib_head.so python -u scripts/compare_builds.py dump gpurun_out/zs_prev.npz
step zs_dump_cur 300 python -u scripts/compare_builds.py dump gpurun_out/zs_cur.npz
step zs_compare 120 python -u scripts/compare_builds.py compare gpurun_out/zs_prev.npz gpurun_out/zs_cur.npz
B="python bench.py --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0"
for cfg in c4 c1k4 d4ic; do
  step zs_head_$cfg 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_head.so $B --config $cfg
  step zs_mfma_$cfg 200 $B --config $cfg
done
step zs_trace_d4ic 200 python -u scripts/phase_trace.py --config d4ic
step zs_suite 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread
kill $HB
