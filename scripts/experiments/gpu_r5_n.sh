#!/bin/bash
# Round 5: GPU suite + smoke on the new defaults (channel-sliced embedder forward, fence-free fork /
# join events, 3-wave k_fac_bwd_s16); per-step kernel timelines of C1(K=4) with and without the split
# lead; the default bench line
source "$(dirname "$0")/../gpu_steps.sh"
step n_suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA --durations=10
step n_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
K="--steps 50 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times --config c1k4 --preheat-s 0"
step n_kt 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/n/kt -o run -- python bench.py $K
f=$(ls gpurun_out/n/kt/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && step n_timeline 60 python scripts/step_timeline.py "$f" --steps 4
REDCLIFF_SPLIT_LEAD=0 step n_kt0 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/n/kt0 -o run -- python bench.py $K
f=$(ls gpurun_out/n/kt0/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && step n_timeline0 60 python scripts/step_timeline.py "$f" --steps 4
rm -rf gpurun_out/n/kt gpurun_out/n/kt0
step n_bench 600 python bench.py
# the merged backward at 3 waves per SIMD (scripts/bin/lib_mw3.so, -DRC_MERGED_WAVES=3): resident at C1(K=4)
M=scripts/bin/lib_mw3.so
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
  for cfg in c1k4 c4 d4ic; do
    step n_${cfg}_base_$rep 200 $B --config $cfg
    REDCLIFF_HIP_LIB=$M step n_${cfg}_mw3_$rep 200 $B --config $cfg
  done
done
REDCLIFF_HIP_LIB=$M step n_mw3_tests 600 python -u -m pytest tests/test_gpu_forked.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -rA
