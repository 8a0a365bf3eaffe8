#!/bin/bash
# Packed-fit kernel trace (R=128 D4IC, 40 epochs): which launches make up validation and GC tracking
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4i
timeout -k 10 300 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 > gpurun_out/r4i/pf.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4i/prof -o pf -- python3 scripts/pack_fit_profile.py --replicas 128 --epochs 40 > gpurun_out/r4i/pf_prof.log 2>&1
