# parity tests + workgroup trace of d4ic (quick iteration loop)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u scripts/phase_trace.py --config d4ic > gpurun_out/trace_d4ic.log 2>&1
