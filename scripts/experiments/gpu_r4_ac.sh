#!/bin/bash
# Round 4 experiment: k_fac_bwd_s16 with the Adam moments requested one block ahead (2 waves/SIMD)
# vs the default (3 waves/SIMD): grid step A/B interleaved, kernel stats (one stream)
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4ac
for i in 1 2; do
step ac_grid_def$i 200 python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2 --settings '[{}]'
step ac_grid_mva$i 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_mvahead.so python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2 --settings '[{}]'
done
step ac_prof_def 200 env REDCLIFF_FORK=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ac/def -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step ac_prof_mva 200 env REDCLIFF_FORK=0 REDCLIFF_HIP_LIB=scripts/bin/lib_mvahead.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ac/mva -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step ac_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pack_fit.py tests/test_gpu_replicas.py
kill $HB
