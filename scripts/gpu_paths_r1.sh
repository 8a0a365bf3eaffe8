#!/bin/bash
# single-fit factor-path / stream variants at D4IC and C1(K=4) (bench windows/s, no CPU leg)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline --replicas 1 --steps 300 --warmup 30"
REDCLIFF_FAC_PATH=mfma timeout -k 10 120 $B > gpurun_out/r1_mfma.log 2>&1 && \
REDCLIFF_FORK=1 timeout -k 10 120 $B > gpurun_out/r1_fork.log 2>&1 && \
timeout -k 10 120 $B > gpurun_out/r1_default.log 2>&1 && \
REDCLIFF_FAC_PATH=mfma timeout -k 10 120 $B --config c1k4 > gpurun_out/r1_c1_mfma.log 2>&1 && \
timeout -k 10 120 $B --config c1k4 > gpurun_out/r1_c1_default.log 2>&1
