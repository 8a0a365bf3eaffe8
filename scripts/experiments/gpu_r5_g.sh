#!/bin/bash
# Round 5: full GPU suite (HipAdam on the generic path, the reverted division forms), smoke, bench line
source "$(dirname "$0")/../gpu_steps.sh"
step g_suite 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=12 -rA
step g_smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step g_bench 600 python bench.py --steps 20 --warmup 5
