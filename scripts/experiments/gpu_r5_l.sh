#!/bin/bash
# Round 5: C1(K=4) single fit with the channel-sliced embedder forward (200 columns per slice): step
# launch-structure knobs, and a rocprofv3 kernel trace for the per-step timeline (gaps between kernels)
source "$(dirname "$0")/../gpu_steps.sh"
export REDCLIFF_EMB_FWD_COLS=200
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times --config c1k4"
for rep in 1 2; do
  step l_base_$rep 200 $B
  REDCLIFF_DEFER=0 step l_defer0_$rep 200 $B
  REDCLIFF_DEFER=2 step l_defer2_$rep 200 $B
  REDCLIFF_MERGE=1 step l_merge1_$rep 200 $B
  REDCLIFF_SPLIT_LEAD=0 step l_split0_$rep 200 $B
  REDCLIFF_FAC_PATH=mfma step l_mfma_$rep 200 $B
done
step l_kt 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/l/kt -o run -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times --config c1k4 --preheat-s 0
f=$(ls gpurun_out/l/kt/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && step l_timeline 60 python scripts/step_timeline.py "$f" --steps 4
rm -rf gpurun_out/l/kt
