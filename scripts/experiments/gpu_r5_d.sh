#!/bin/bash
# Round 5: the driver's bench line (with the reference-grid leg and the one-stream grid roofline), grid-only
# kernel stats at R = 128 (one stream and forked), HBM counter passes (grid and single fit), the copy
# attribution of the packed fit
source "$(dirname "$0")/../gpu_steps.sh"
mkdir -p gpurun_out/d
S="python bench.py --steps 30 --warmup 5 --preheat-s 0 --no-cpu-baseline --no-north-star --no-kernel-times --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0"
G="python scripts/grid_step.py --replicas 128 --steps 3"
F="--kernel-include-regex k_ --output-format csv"
step d_bench 600 python bench.py --steps 20 --warmup 5
REDCLIFF_FORK=0 step d_gstats1 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/d/gstats1 -o run -- python scripts/grid_step.py --replicas 128 --steps 20
step d_gstats2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/d/gstats2 -o run -- python scripts/grid_step.py --replicas 128 --steps 20
step d_gfetch 150 rocprofv3 --pmc FETCH_SIZE $F -d gpurun_out/d/pmc_g_fetch -o run -- $G
step d_gwrite 150 rocprofv3 --pmc WRITE_SIZE $F -d gpurun_out/d/pmc_g_write -o run -- $G
step d_fetch 150 rocprofv3 --pmc FETCH_SIZE $F -d gpurun_out/d/pmc_s_fetch -o run -- $S
step d_write 150 rocprofv3 --pmc WRITE_SIZE $F -d gpurun_out/d/pmc_s_write -o run -- $S
step d_copies 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/d/ca -o run -- python scripts/copy_attribution.py --replicas 128 --epochs 40
