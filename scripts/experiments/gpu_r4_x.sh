#!/bin/bash
# Round 4: k_fac_bwd_s16 phases alone (timing experiments: contraction only / Adam stream only)
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4x
step x_tree 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4x/tree -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step x_nomfma 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_s16_nompfma.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4x/nomfma -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step x_noepi 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_s16_noepi.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4x/noepi -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
kill $HB
