cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_generic.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_generic.log 2>&1
