#!/bin/bash
# recompute debug build: print activations whose recomputation differs from the forward's
source "$(dirname "$0")/../gpu_steps.sh"
export REDCLIFF_FAC_PATH=mfma REDCLIFF_FORK=0 COMPARE_EPOCHS=1 COMPARE_BATCHES=2
REDCLIFF_HIP_LIB=exp/lib_dbg.so step d_dbg 200 python -u scripts/compare_builds.py dump gpurun_out/dbg.npz
grep -c RECOMP gpurun_out/d_dbg.log; grep RECOMP gpurun_out/d_dbg.log | head -20
