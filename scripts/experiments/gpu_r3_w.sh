#!/bin/bash
# Round 3: embedder forward deeper fc1 prefetch (graph convolution back to the vector form) -- full GPU
# suite, D4IC and TST single-fit bench lines, D4IC phase timeline, kernel stats.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step w_suite 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --durations=5
step w_d4ic 300 python bench.py --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step w_c4 300 python bench.py --config c4 --steps 200 --warmup 20 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step w_c1k4 300 python bench.py --config c1k4 --steps 200 --warmup 20 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0
step w_trace 200 python -u scripts/phase_trace.py --config d4ic
kill $HB
