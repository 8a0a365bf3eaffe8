#!/bin/bash
# Round 3: where the TST-shaped single fit and the data-parallel update spend their time --
# workgroup timeline of the c4 (TST) step, kernel stats of scripts/dp_profile.py at B=128.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step x_trace_c4 200 python -u scripts/phase_trace.py --config c4
step x_dp 300 python -u scripts/dp_profile.py --batch 128 --steps 200
step x_dp_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/x_dp_prof -o dp -- python -u scripts/dp_profile.py --batch 128 --steps 200
kill $HB
