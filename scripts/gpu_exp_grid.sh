#!/bin/bash
# packed-grid experiment: embedder-backward LDS sub-block size (occupancy) at R = 32
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline --steps 30 --warmup 5 --replicas 32 --grid-steps 100"
timeout -k 10 200 $B > gpurun_out/g_base.log 2>&1 || exit 1
REDCLIFF_HIP_LIB=exp/lib_bc8.so timeout -k 10 200 $B > gpurun_out/g_bc8.log 2>&1 || exit 1
REDCLIFF_HIP_LIB=exp/lib_bc4.so timeout -k 10 200 $B > gpurun_out/g_bc4.log 2>&1 || exit 1
