#!/bin/bash
# k_fac_bwd_mfma occupancy variants on the R = 32 grid: epilogue prefetch (p) vs none (np), waves/EU hint
source "$(dirname "$0")/../gpu_steps.sh"
G="python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-north-star --fit-replicas 0 --grid-steps 50 --replicas 32"
for v in fb_p1 fb_np1 fb_np3 fb_p1 fb_np1 fb_np3; do
  REDCLIFF_HIP_LIB=exp/lib_$v.so step $v 200 $G
  grep '^{' gpurun_out/$v.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); g=d['grid_search']; print('$v', g['windows_per_s'], g['ms_per_step'], g['roofline']['kernel_avg_us']['fac_bwd'])"
done
