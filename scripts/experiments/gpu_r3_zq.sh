#!/bin/bash
# Round 3: vector factor backward's activation recompute and dW0 tile on 16x16x4 matrix-core tiles
# (same fmaf chains) -- bitwise comparison against the committed build, A/B interleaved, suite
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step zq_dump_prev 300 env REDCLIFF_HIP_LIB=scripts/bin/lib_head.so python -u scripts/compare_builds.py dump gpurun_out/zq_prev.npz
step zq_dump_cur 300 python -u scripts/compare_builds.py dump gpurun_out/zq_cur.npz
step zq_compare 120 python -u scripts/compare_builds.py compare gpurun_out/zq_prev.npz gpurun_out/zq_cur.npz
B="python bench.py --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0"
for cfg in c4 c1k4 d4ic; do
  step zq_head_$cfg 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_head.so $B --config $cfg
  step zq_mfma_$cfg 200 $B --config $cfg
done
step zq_trace_c4 200 python -u scripts/phase_trace.py --config c4
step zq_suite 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread
kill $HB
