cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in d4ic c5; do timeout -k 10 120 python -u scripts/phase_trace.py --config $c > gpurun_out/trace_$c.log 2>&1 || exit 1; done
