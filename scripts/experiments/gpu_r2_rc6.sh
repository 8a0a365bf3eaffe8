#!/bin/bash
# recompute build vs previous: 1, 2 and 3 batches of the acclimate epoch (params + Adam moments)
source "$(dirname "$0")/../gpu_steps.sh"
export REDCLIFF_FAC_PATH=mfma REDCLIFF_FORK=0 COMPARE_EPOCHS=1
for nb in 1 2 3; do
  export COMPARE_BATCHES=$nb
  REDCLIFF_HIP_LIB=exp/lib_prev.so step d_prev 200 python -u scripts/compare_builds.py dump gpurun_out/p$nb.npz
  step d_cur 200 python -u scripts/compare_builds.py dump gpurun_out/c$nb.npz
done
