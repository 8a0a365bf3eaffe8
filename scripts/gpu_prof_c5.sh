cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_c5 -o run -- python bench.py --config c5 --no-cpu-baseline --steps 20 --warmup 3 --replicas 1 --no-kernel-times > gpurun_out/kt_c5.log 2>&1
