#!/bin/bash
# Round 5: the multi-sub-block embedder backward (B = 512 data-parallel shard steps) back to its
# session-start register budget (the one-round fc2 staging, the batched dL/dw rounds and the early
# BatchNorm loads spilled it into 30 accumulation registers: 256 + 32 registers, one wave per SIMD,
# 212 -> 363 us).  Data-parallel leg and single fits against the previous build, kernel stats of
# the data-parallel leg, the data-parallel and fit tests, then the whole GPU suite.
source "$(dirname "$0")/../gpu_steps.sh"
P=scripts/bin/lib_prev_r5o.so
D="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
  REDCLIFF_HIP_LIB=$P step ao_prev_dp_$rep 200 $D
  step ao_cur_dp_$rep 200 $D
done
step ao_stats 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ao/cur -o run -- $D
rm -f gpurun_out/ao/*/run_kernel_trace.csv
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for cfg in c1k4 c4 d4ic; do
  REDCLIFF_HIP_LIB=$P step ao_prev_${cfg} 200 $B --config $cfg
  step ao_cur_${cfg} 200 $B --config $cfg
done
step ao_suite 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x
