#!/bin/bash
# Round 6 tree: the driver's round-end sequence (GPU suite, smoke, bench line).
source "$(dirname "$0")/../gpu_steps.sh"
step e_suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA --durations=15
step e_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step e_bench 600 python bench.py
