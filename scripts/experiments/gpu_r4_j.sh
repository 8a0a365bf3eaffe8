#!/bin/bash
# Round 4: adjacency dS sums in one load round + NR=1 tail (bits vs HEAD build, A/B single fits),
# packed-fit kernel trace at R=128
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4j
step j_dump_prev 300 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python -u scripts/compare_builds.py dump gpurun_out/r4j/prev.npz
step j_dump_cur 300 python -u scripts/compare_builds.py dump gpurun_out/r4j/cur.npz
step j_compare 120 python -u scripts/compare_builds.py compare gpurun_out/r4j/prev.npz gpurun_out/r4j/cur.npz
step j_ab_prev1 240 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python -u scripts/ab_single.py --tag prev
step j_ab_cur1 240 python -u scripts/ab_single.py --tag cur
step j_ab_nr4 240 env REDCLIFF_HIP_LIB=scripts/bin/lib_nr4.so python -u scripts/ab_single.py --tag flat_nr4
step j_ab_prev2 240 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python -u scripts/ab_single.py --tag prev
step j_ab_cur2 240 python -u scripts/ab_single.py --tag cur
step j_forked 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_forked.py
step j_pf 300 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40
step j_pf_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4j/prof -o pf -- python3 scripts/pack_fit_profile.py --replicas 128 --epochs 40
kill $HB
