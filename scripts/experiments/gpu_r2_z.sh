#!/bin/bash
# packed-grid path check: matrix-core (default at R >= 8) vs vector factor path; R sweep
source "$(dirname "$0")/../gpu_steps.sh"
G="python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-north-star --fit-replicas 0 --grid-steps 50"
step g_mfma32 200 $G --replicas 32
REDCLIFF_FAC_PATH=vector step g_vec32 200 $G --replicas 32
step g_mfma64 200 $G --replicas 64
step g_mfma16 200 $G --replicas 16
for f in g_mfma32 g_vec32 g_mfma64 g_mfma16; do grep '^{' gpurun_out/$f.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); g=d['grid_search']; print('$f', g['replicas_per_gpu'], g['windows_per_s'], g['ms_per_step'], g['roofline']['kernel_avg_us'])"; done
