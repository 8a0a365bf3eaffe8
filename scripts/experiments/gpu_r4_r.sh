#!/bin/bash
# Round 4: fewer, longer waves in the evaluation kernels (GC norms one wave per network, cosine
# values / GC dots two windows / samples per wave): kernel stats, bitwise fit records, profile
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4r
step r_dump_cur 300 python -u scripts/compare_fits.py dump gpurun_out/r4r/fcur.npz
step r_eval_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4r/prof -o ev -- python3 scripts/eval_kernels.py --reps 10
step r_pf_split 400 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --host-split
kill $HB
