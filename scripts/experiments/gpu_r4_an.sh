#!/bin/bash
# Round 4: XCD-aware tile order of the GEMM core (every tile of one replica / slice on one XCD):
# bitwise packed fits, in-process interleaved A/B against dispatch order, HBM fetch per GEMM
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4an
step an_dump8 300 env COMPARE_FITS_R=8 python -u scripts/compare_fits.py dump gpurun_out/r4an/fcur8.npz
step an_sweep 400 python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 4 --settings '[{}, {"REDCLIFF_GEMM_XCD": "0"}]'
step an_sweep_r32 300 python -u scripts/grid_sweep.py --replicas 32 --steps 40 --rounds 4 --settings '[{}, {"REDCLIFF_GEMM_XCD": "0"}]'
step an_pmc_on 120 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r4an/pon -o f -- python3 scripts/grid_step.py --replicas 128 --steps 3
step an_pmc_off 120 env REDCLIFF_GEMM_XCD=0 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r4an/poff -o f -- python3 scripts/grid_step.py --replicas 128 --steps 3
step an_prof_on 200 env REDCLIFF_FORK=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4an/son -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step an_prof_off 200 env REDCLIFF_FORK=0 REDCLIFF_GEMM_XCD=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4an/soff -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
step an_tests 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_generic.py tests/test_gpu_replicas.py tests/test_gpu_parity.py
kill $HB
