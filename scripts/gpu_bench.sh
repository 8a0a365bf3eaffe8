# bench (d4ic + grid, c5) and rocprofv3 kernel-trace summary of the d4ic bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --steps 50 --warmup 5 --replicas 1 > gpurun_out/bench_c5.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o run -- python bench.py --no-cpu-baseline --steps 300 --warmup 30 --replicas 1 > gpurun_out/kt.log 2>&1
