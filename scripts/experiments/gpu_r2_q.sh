#!/bin/bash
# host-side cProfile of the packed D4IC fit
source "$(dirname "$0")/../gpu_steps.sh"
step r2_packprof_cprof 300 python -u scripts/pack_fit_profile.py --config d4ic --cprofile
