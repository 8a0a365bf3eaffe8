#!/bin/bash
# single-fit experiment: windows per embedder-forward workgroup (D4IC and C1(K=4))
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for sb in 1 2 4; do
  REDCLIFF_EMB_SB=$sb timeout -k 10 200 python -u bench.py --no-cpu-baseline --replicas 1 > gpurun_out/d4ic_sb$sb.log 2>&1 || exit 1
  REDCLIFF_EMB_SB=$sb timeout -k 10 200 python -u bench.py --config c1k4 --no-cpu-baseline --replicas 1 > gpurun_out/c1k4_sb$sb.log 2>&1 || exit 1
done
