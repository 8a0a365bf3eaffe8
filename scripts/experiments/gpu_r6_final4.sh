#!/bin/bash
# Round 6 final tree (+ k_lemb_dhead operands requested up front; k_lemb_head 4 windows per wave, k_emb_final parameters with the
# gradients): GPU suite, smoke, default bench line, kernel-trace summaries of the R = 128 grids
# (factor chain on one stream) at D4IC and TST.
source "$(dirname "$0")/../gpu_steps.sh"
step f4_suite 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA --durations=15
step f4_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step f4_bench 600 python bench.py
for cfg in d4ic c4; do
  REDCLIFF_FORK=0 step f4_gstats_$cfg 240 timeout -s KILL 220 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f4/$cfg -o run -- python scripts/grid_step.py --replicas 128 --steps 20 --config $cfg
done
rm -f gpurun_out/f4/*/run_kernel_trace.csv
