#!/bin/bash
# Round 5: which kernels of the data-parallel leg (TST shape, B = 512 shard steps, RC_GRAD_ONLY) got
# slower between the session-start build and the current one: kernel stats of the same bench command.
source "$(dirname "$0")/../gpu_steps.sh"
D="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --ref-grid-epochs 0 --no-kernel-times"
step an_cur 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/an/cur -o run -- $D
REDCLIFF_HIP_LIB=scripts/bin/lib_start_r5s.so step an_start 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/an/start -o run -- $D
rm -f gpurun_out/an/*/run_kernel_trace.csv
