#!/bin/bash
# one acclimate step (factor backward only), single stream, matrix-core path: prev vs current
source "$(dirname "$0")/../gpu_steps.sh"
export REDCLIFF_FAC_PATH=mfma REDCLIFF_FORK=0 COMPARE_EPOCHS=1 COMPARE_ONE_BATCH=1
step rc_dump_prev 200 python -u scripts/compare_builds.py dump gpurun_out/prev1.npz
REDCLIFF_HIP_LIB=exp/lib_rc.so step rc_dump_cur 200 python -u scripts/compare_builds.py dump gpurun_out/cur1.npz
