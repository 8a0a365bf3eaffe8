cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_data_parallel.py tests/test_gpu_replicas.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_dp.log 2>&1
