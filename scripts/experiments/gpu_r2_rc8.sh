#!/bin/bash
# output-layer gradients of network 0 per step: previous build (mix) vs recompute build (bwd)
source "$(dirname "$0")/../gpu_steps.sh"
export REDCLIFF_FAC_PATH=mfma REDCLIFF_FORK=0 COMPARE_EPOCHS=1 COMPARE_BATCHES=2
REDCLIFF_HIP_LIB=exp/lib_pdbg.so step d_pdbg 200 python -u scripts/compare_builds.py dump gpurun_out/x1.npz
REDCLIFF_HIP_LIB=exp/lib_dbg.so step d_dbg 200 python -u scripts/compare_builds.py dump gpurun_out/x2.npz
rm -f gpurun_out/x1.npz gpurun_out/x2.npz
