#!/bin/bash
# Round 4: s16 forward with 4 tiles per pass vs 2 (grid step kernel stats, bits via the replica tests)
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4y
step y_t4 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4y/t4 -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step y_t2 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_fwd2.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4y/t2 -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step y_t4b 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4y/t4b -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step y_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py
kill $HB
