#!/bin/bash
source "$(dirname "$0")/../gpu_steps.sh"
step r2_c5 600 python -u -m pytest tests/test_gpu_parity.py -v -s -k stress --timeout 500 --timeout-method thread
