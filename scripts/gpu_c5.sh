cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"
for c in d4ic c5; do timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; break; }; done
