#!/bin/bash
# Round 5: split-lead records merged into the embedder backward's launch (k_bwd_lead_emb, default
# for split-lead steps; REDCLIFF_LEAD_EMB=0 keeps the records launch).  Bitwise test, single-fit
# steps with and without it (C1(K=4) splits by default; TST forced split too), the step timeline,
# phase trace, the forked / golden suites.
source "$(dirname "$0")/../gpu_steps.sh"
T="python -u -m pytest -v --timeout 300 --timeout-method thread -rA"
step al_test 300 $T tests/test_gpu_forked.py -k "lead_records or split_lead or kernel_completed"
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
  REDCLIFF_LEAD_EMB=0 step al_off_c1k4_$rep 200 $B --config c1k4
  step al_on_c1k4_$rep 200 $B --config c1k4
  REDCLIFF_SPLIT_LEAD=1 REDCLIFF_LEAD_EMB=0 step al_off_c4_$rep 200 $B --config c4
  REDCLIFF_SPLIT_LEAD=1 step al_on_c4_$rep 200 $B --config c4
  step al_def_c4_$rep 200 $B --config c4
done
step al_trace_c1k4 200 python scripts/phase_trace.py --config c1k4
K="--steps 50 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times --config c1k4 --preheat-s 0"
step al_kt 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/al/kt -o run -- python bench.py $K
f=$(ls gpurun_out/al/kt/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && step al_timeline 60 python scripts/step_timeline.py "$f" --steps 3
rm -rf gpurun_out/al/kt
step al_suite 600 $T tests/test_gpu_forked.py tests/test_gpu_fit_golden.py tests/test_gpu_replicas.py tests/test_gpu_parity.py
