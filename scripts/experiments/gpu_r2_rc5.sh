#!/bin/bash
# where the recompute build departs from the previous one: single stream 4 epochs / forked 1 step
source "$(dirname "$0")/../gpu_steps.sh"
export REDCLIFF_FAC_PATH=mfma
for mode in "0 0,1,2,3 " "1 1 1" "0 1,2 " "0 1 "; do
  set -- $mode
  export REDCLIFF_FORK=$1 COMPARE_EPOCHS=$2
  if [ -n "$3" ]; then export COMPARE_ONE_BATCH=1; else unset COMPARE_ONE_BATCH; fi
  REDCLIFF_HIP_LIB=exp/lib_prev.so step d_prev 200 python -u scripts/compare_builds.py dump gpurun_out/p.npz
  step d_cur 200 python -u scripts/compare_builds.py dump gpurun_out/c.npz
  echo "fork=$1 epochs=$2 onebatch=$3: $(python -u scripts/compare_builds.py compare gpurun_out/p.npz gpurun_out/c.npz | tail -1)"
done
rm -f gpurun_out/p.npz gpurun_out/c.npz
