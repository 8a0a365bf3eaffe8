#!/bin/bash
# Round 3: embedder-backward node staging -- dL/dw partial rounds issued together (p <= 16), BatchNorm
# affine terms staged with the windows -- full suite, single-fit bench lines, TST timeline.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step zf_suite 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --durations=5
step zf_c4 300 python bench.py --config c4 --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step zf_c1k4 300 python bench.py --config c1k4 --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step zf_d4ic 300 python bench.py --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step zf_trace_c4 200 python -u scripts/phase_trace.py --config c4
kill $HB
