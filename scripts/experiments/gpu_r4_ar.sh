#!/bin/bash
# Round 4: per-kernel breakdown of the north-star C1(K=4) and TST single fits
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4ar
step ar_c1k4 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ar/c1k4 -o s -- python3 scripts/ab_single.py --tag c1k4 --configs c1k4
step ar_c4 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ar/c4 -o s -- python3 scripts/ab_single.py --tag c4 --configs c4
step ar_d4ic 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ar/d4ic -o s -- python3 scripts/ab_single.py --tag d4ic --configs d4ic
kill $HB
