#!/bin/bash
# Round 4: XCD-aware workgroup order in k_fac_mix and the short-contraction factor kernels
# (every workgroup of one replica on one XCD): bitwise packed fits, in-process A/B, HBM fetch
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4ap
step ap_dump8 300 env COMPARE_FITS_R=8 python -u scripts/compare_fits.py dump gpurun_out/r4ap/fcur8.npz
step ap_sweep 500 python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 4 --settings '[{}, {"REDCLIFF_MIX_XCD": "0", "REDCLIFF_S16_XCD": "0"}, {"REDCLIFF_S16_XCD": "0"}]'
step ap_pmc_on 120 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_ --output-format csv -d gpurun_out/r4ap/pon -o f -- python3 scripts/grid_step.py --replicas 128 --steps 3
step ap_pmc_off 120 env REDCLIFF_MIX_XCD=0 REDCLIFF_S16_XCD=0 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_ --output-format csv -d gpurun_out/r4ap/poff -o f -- python3 scripts/grid_step.py --replicas 128 --steps 3
step ap_prof_on 200 env REDCLIFF_FORK=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ap/son -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step ap_prof_off 200 env REDCLIFF_FORK=0 REDCLIFF_MIX_XCD=0 REDCLIFF_S16_XCD=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ap/soff -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step ap_tests 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_replicas.py tests/test_gpu_pack_fit.py tests/test_gpu_forked.py
kill $HB
