#!/bin/bash
# Round 6: the GPU suite on the final tree.
source "$(dirname "$0")/../gpu_steps.sh"
step y_suite 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA --durations=15
step y_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
