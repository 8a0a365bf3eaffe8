#!/bin/bash
# Round 3: merged backward with the non-lead factor workgroups held until the leads publish
# (REDCLIFF_LEAD_FIRST) -- A/B interleaved at D4IC, timeline; DP update with 4 elements per thread
source "$(dirname "$0")/../gpu_steps.sh"
B="python bench.py --steps 300 --warmup 30 --replicas 1 --fit-replicas 0 --no-north-star --no-cpu-baseline --dp-leg-batch 0"
for rep in 1 2; do
  step zo_off_$rep 200 $B --config d4ic
  step zo_on_$rep 200 env REDCLIFF_LEAD_FIRST=1 $B --config d4ic
done
step zo_trace_on 200 env REDCLIFF_LEAD_FIRST=1 python -u scripts/phase_trace.py --config d4ic
step zo_dp 200 python -u scripts/dp_profile.py --batch 128 --steps 200
step zo_merged_tests 300 env REDCLIFF_LEAD_FIRST=1 python -u -m pytest tests/test_gpu_forked.py tests/test_gpu_status.py -v --timeout 120 --timeout-method thread
