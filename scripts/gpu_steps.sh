#!/bin/bash
# Helper for GPU-box command files: step NAME SECONDS CMD... runs CMD under its own time limit,
# logs to gpurun_out/NAME.log, and ends the whole call on a time limit, abort or crash (no
# further GPU step after a fault); an ordinary non-zero exit (a failing test) is recorded and
# the next step still runs.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
: > gpurun_out/steps.txt
step() {
  local name=$1 secs=$2
  shift 2
  echo "== $name: $*" | tee -a gpurun_out/steps.txt
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.txt
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then
    echo "== stopping after $name (rc=$rc)" | tee -a gpurun_out/steps.txt
    exit $rc
  fi
  return 0
}
