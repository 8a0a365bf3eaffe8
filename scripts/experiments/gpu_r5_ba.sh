#!/bin/bash
# Round 5 final tree, the driver's own round-end sequence: GPU suite, smoke, bench line.
source "$(dirname "$0")/../gpu_steps.sh"
step ba_suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA --durations=10
step ba_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step ba_bench 600 python bench.py
