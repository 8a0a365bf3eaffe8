#!/bin/bash
# replica-count sweep of the current build: packed grid step and whole-fit fits/hour
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
for R in 32 64 128; do
  step sw_$R 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-north-star --no-kernel-times --grid-steps 50 --replicas $R --fit-replicas $R
  grep '^{' gpurun_out/sw_$R.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); g=d['grid_search']; f=d['fits_per_hour']; print('R=$R grid', g['windows_per_s'], g['ms_per_step'], 'fits/h', f['value'], f['seconds'])"
done
kill $HB
