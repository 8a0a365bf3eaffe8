#!/bin/bash
# Timing experiments: the C5 bench with each exp/lib_*.so variant.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in exp/lib_*.so; do
  n=$(basename $v .so)
  REDCLIFF_HIP_LIB=$PWD/$v timeout -k 10 200 python -u bench.py --config c5 --no-cpu-baseline --steps 30 --warmup 3 --replicas 1 > gpurun_out/exp_$n.log 2>&1 || exit 1
done
