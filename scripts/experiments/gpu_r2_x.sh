#!/bin/bash
# kernel trace of the packed D4IC fit: where the GPU time of an epoch goes
source "$(dirname "$0")/../gpu_steps.sh"
step r2_packtrace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/packtrace -o run -- python scripts/pack_fit_profile.py --config d4ic
