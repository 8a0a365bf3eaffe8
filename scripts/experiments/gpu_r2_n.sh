#!/bin/bash
# Session re-entry check of the committed build: whole GPU suite, smoke, the driver's bench
# command, and the kernel-trace summary of the same bench command.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step r2_suite 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
step r2_smoke 200 python -u __graft_entry__.py smoke
step r2_bench 400 python -u bench.py --steps 20 --warmup 5
step r2_kstats 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kstats -o run -- python bench.py --no-cpu-baseline --steps 20 --warmup 5 --replicas 1 --fit-replicas 0 --no-north-star
kill $HB
