#!/bin/bash
# k_fac_bwd_mfma: waves/EU 4 on the grid; C5 single fit with each variant
source "$(dirname "$0")/../gpu_steps.sh"
G="python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-north-star --fit-replicas 0 --grid-steps 50 --replicas 32"
C="python -u bench.py --config c5 --steps 30 --warmup 5 --no-cpu-baseline --no-north-star --fit-replicas 0 --replicas 1"
for v in fb_np4 fb_np3; do
  REDCLIFF_HIP_LIB=exp/lib_$v.so step $v 200 $G
  grep '^{' gpurun_out/$v.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); g=d['grid_search']; print('$v grid', g['windows_per_s'], g['ms_per_step'], g['roofline']['kernel_avg_us']['fac_bwd'])"
done
for v in fb_p1 fb_np3 fb_p1 fb_np3; do
  REDCLIFF_HIP_LIB=exp/lib_$v.so step c5_$v 200 $C
  grep '^{' gpurun_out/c5_$v.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$v c5', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])"
done
