#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration for 4 B/lane and 16 B/lane streams, then the driver's bench
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step r2_calib_fetch 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib_fetch -o run -- scripts/bin/fetch_calib
step r2_calib_write 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib_write -o run -- scripts/bin/fetch_calib
step r2_bench 400 python -u bench.py --steps 20 --warmup 5
kill $HB
