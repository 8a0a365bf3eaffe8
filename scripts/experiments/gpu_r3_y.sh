#!/bin/bash
# Round 3: split-lead step (factor-lead records in their own launch, factor update on the second
# stream beside the embedder backward) -- full GPU suite, TST / C1(K=4) / D4IC bench lines, TST
# timeline, data-parallel update profile.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step y_suite 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --durations=5
step y_c4 300 python bench.py --config c4 --steps 200 --warmup 20 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step y_c1k4 300 python bench.py --config c1k4 --steps 200 --warmup 20 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step y_d4ic 300 python bench.py --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step y_trace_c4 200 python -u scripts/phase_trace.py --config c4
step y_dp 300 python -u scripts/dp_profile.py --batch 128 --steps 200
kill $HB
