#!/bin/bash
# Factor-path comparison on the bench configs: single fit and packed grid search.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -k "three_phases" > gpurun_out/pytest_paths.log 2>&1 || exit 1
for path in vector mfma; do
  REDCLIFF_FAC_PATH=$path timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 200 --warmup 20 --replicas 32 --grid-steps 50 > gpurun_out/bench_path_$path.log 2>&1 || exit 1
done
