#!/bin/bash
# bitwise dumps (matrix-core path) of the previous and the current build, kept for analysis
source "$(dirname "$0")/../gpu_steps.sh"
export REDCLIFF_FAC_PATH=mfma
REDCLIFF_HIP_LIB=exp/lib_prev.so step rc_dump_prev 200 python -u scripts/compare_builds.py dump gpurun_out/prev.npz
step rc_dump_cur 200 python -u scripts/compare_builds.py dump gpurun_out/cur.npz
