#!/bin/bash
# Round 2, first GPU call: forked-vs-single-stream bitwise tests under guard bands, the race
# probe, then the whole GPU suite.
source "$(dirname "$0")/../gpu_steps.sh"
step r2_forked 300 python -u -m pytest tests/test_gpu_forked.py -x -v --timeout 120 --timeout-method thread
step r2_race_probe 400 python -u scripts/race_probe.py
step r2_gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
