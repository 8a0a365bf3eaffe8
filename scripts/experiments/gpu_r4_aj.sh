#!/bin/bash
# Round 4: accumulator-layout factor backward variants, interleaved grid A/B and kernel stats:
# prev (lane-linear epilogue, HEAD), late4 (operands after the contraction, 4 waves),
# e3 (operands at the block start, 3 waves), e4 (at the block start, 4 waves, small spill)
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/r4aj
for i in 1 2; do
for v in prev late4 e3 e4; do
step aj_grid_${v}$i 200 env REDCLIFF_HIP_LIB=scripts/bin/lib_$v.so python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 2 --settings '[{}]'
done
done
for v in prev late4 e3 e4; do
step aj_prof_$v 200 env REDCLIFF_FORK=0 REDCLIFF_HIP_LIB=scripts/bin/lib_$v.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4aj/$v -o g -- python3 scripts/grid_step.py --replicas 128 --steps 20
done
kill $HB
