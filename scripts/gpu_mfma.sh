cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k "three_phases or stress" > gpurun_out/pytest_mfma.log 2>&1
echo "pytest rc=$?"
timeout -k 10 200 python -u bench.py --config c5 --no-cpu-baseline --steps 50 --warmup 5 --replicas 1 > gpurun_out/bench_c5.log 2>&1
