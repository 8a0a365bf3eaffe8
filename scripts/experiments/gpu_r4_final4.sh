#!/bin/bash
# Round 4, final tree (after the k_emb_final loads and the LDS loop unrolls): full GPU suite, smoke, the driver's default bench line, its kernel stats,
# HBM counter passes (single fit and R=128 grid) for the roofline traffic field
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
mkdir -p gpurun_out/f4
S="python bench.py --steps 30 --warmup 5 --preheat-s 0 --no-cpu-baseline --no-north-star --no-kernel-times --replicas 1 --fit-replicas 0 --dp-leg-batch 0"
G="python scripts/grid_step.py --replicas 128 --steps 3"
F="--kernel-include-regex k_ --output-format csv"
step f4_suite 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread --durations=5
step f4_smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step f4_bench 600 python bench.py --steps 20 --warmup 5
step f4_fetch 150 rocprofv3 --pmc FETCH_SIZE $F -d gpurun_out/f4/pmc_s_fetch -o run -- $S
step f4_write 150 rocprofv3 --pmc WRITE_SIZE $F -d gpurun_out/f4/pmc_s_write -o run -- $S
step f4_gfetch 150 rocprofv3 --pmc FETCH_SIZE $F -d gpurun_out/f4/pmc_g_fetch -o run -- $G
step f4_gwrite 150 rocprofv3 --pmc WRITE_SIZE $F -d gpurun_out/f4/pmc_g_write -o run -- $G
step f4_stats 500 rocprofv3 --kernel-trace --stats --kernel-include-regex k_ --output-format csv -d gpurun_out/f4/stats -o run -- python bench.py --no-cpu-baseline --steps 100 --warmup 10
step f4_bench2 600 python bench.py --steps 20 --warmup 5
kill $HB
