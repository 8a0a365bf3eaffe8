#!/bin/bash
# Round 5: kernel-completed fork / join events on the packed grid's forked matrix-core chain
# (REDCLIFF_EXT_EVENT=0: event-record packets), R = 32 / 128 grid steps; forked-step bitwise tests
source "$(dirname "$0")/../gpu_steps.sh"
step u_tests 600 python -u -m pytest tests/test_gpu_forked.py tests/test_gpu_large_pack.py -v --timeout 300 --timeout-method thread -rA
for R in 32 128; do
  step u_sweep_$R 400 python scripts/grid_sweep.py --replicas $R --steps 50 --rounds 3 --settings '[{},{"REDCLIFF_EXT_EVENT":"0"}]'
done
step u_fits 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-north-star --replicas 1 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times
REDCLIFF_EXT_EVENT=0 step u_fits0 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-north-star --replicas 1 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times
