#!/bin/bash
# Round 5, first call: GPU suite (ABI 9 factor forward, the R = 128 pack tests), smoke, the driver's bench line
source "$(dirname "$0")/../gpu_steps.sh"
step r5a_suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=8 -rA
step r5a_smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step r5a_bench 600 python bench.py --steps 20 --warmup 5
