#!/bin/bash
# Round 3: LDS-staged 16x16x4 short-contraction factor kernels (16-unit blocks), windowed embedder
# with 4 windows per workgroup; suites that pin them, grid A/B + kernel trace, bench line.
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step f_tests 700 python -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_parity.py tests/test_gpu_autograd.py tests/test_gpu_fit_modes.py tests/test_gpu_status.py tests/test_gpu_forked.py tests/test_gpu_pack_fit.py tests/test_gpu_fit_golden.py tests/test_gpu_data_parallel.py -v --timeout 300 --timeout-method thread --durations=15
step f_grid_prev 200 env REDCLIFF_FAC_SHORT=0 REDCLIFF_EMB_WIN=0 python -u scripts/grid_step.py --replicas 128 --steps 20
step f_grid 200 python -u scripts/grid_step.py --replicas 128 --steps 20
step f_kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_grid_f -o run -- python scripts/grid_step.py --replicas 128 --steps 20
step f_bench 500 python -u bench.py --steps 200 --warmup 20
kill $HB
