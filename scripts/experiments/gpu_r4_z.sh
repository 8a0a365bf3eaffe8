#!/bin/bash
# Round 4: k_fac_mix operands in one round of loads: bitwise (fit records, training states) vs
# the HEAD build, grid step A/B interleaved, packed-fit A/B
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4z
step z_dump_cur 300 python -u scripts/compare_fits.py dump gpurun_out/r4z/fcur.npz
step z_bdump_prev 300 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python -u scripts/compare_builds.py dump gpurun_out/r4z/bprev.npz
step z_bdump_cur 300 python -u scripts/compare_builds.py dump gpurun_out/r4z/bcur.npz
step z_bcompare 120 python -u scripts/compare_builds.py compare gpurun_out/r4z/bprev.npz gpurun_out/r4z/bcur.npz
for i in 1 2; do
step z_grid_cur$i 200 python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2 --settings '[{}]'
step z_grid_prev$i 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2 --settings '[{}]'
done
step z_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4z/prof -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
kill $HB
