#!/bin/bash
# Packed grid-search throughput at several replica counts (D4IC) + the factor-path parity tests.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_replicas.py -m gpu -q --timeout 200 --timeout-method thread -k "three_phases or stress or replicas" > gpurun_out/pytest_paths.log 2>&1 || exit 1
for R in 32 64 128; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-kernel-times --steps 20 --warmup 5 --replicas $R --grid-steps 30 > gpurun_out/bench_grid_$R.log 2>&1 || exit 1
done
bash scripts/gpu_prof_grid.sh
