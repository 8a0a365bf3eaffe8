#!/bin/bash
# Round 4 experiment: fc1 weights three column steps ahead (4 buffers, 1 wave/SIMD) vs two (3
# buffers): bits (single fits on the vector path) and single-fit A/B, interleaved
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4ag
step ag_dump3 300 python -u scripts/compare_builds.py dump gpurun_out/r4ag/b3.npz
step ag_dump4 300 env REDCLIFF_HIP_LIB=scripts/bin/lib_fc1b4.so python -u scripts/compare_builds.py dump gpurun_out/r4ag/b4.npz
step ag_cmp 120 python -u scripts/compare_builds.py compare gpurun_out/r4ag/b3.npz gpurun_out/r4ag/b4.npz
for i in 1 2; do
step ag_b3_$i 240 python -u scripts/ab_single.py --tag bufs3
step ag_b4_$i 240 env REDCLIFF_HIP_LIB=scripts/bin/lib_fc1b4.so python -u scripts/ab_single.py --tag bufs4
done
kill $HB
