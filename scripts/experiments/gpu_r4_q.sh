#!/bin/bash
# Round 4: evaluation launches in isolation (events, kernel stats, SQ counters), bitwise fit
# records (compared with the round-start build's dump in the build container), pack-fit profile
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4q
step q_dump_cur 300 python -u scripts/compare_fits.py dump gpurun_out/r4q/fcur.npz
step q_eval 300 python -u scripts/eval_kernels.py
step q_eval_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4q/prof -o ev -- python3 scripts/eval_kernels.py --reps 10
step q_eval_pmc 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU --output-format csv -d gpurun_out/r4q/pmc -o ev -- python3 scripts/eval_kernels.py --reps 3
step q_tests 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pack_fit.py tests/test_gpu_fit_golden.py
step q_pf_split 400 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40 --host-split
kill $HB
