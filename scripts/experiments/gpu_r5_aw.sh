#!/bin/bash
# Round 5: every embedder product on the (register-capped) wave core against the default per-product
# choice: per-kernel traces of the R = 128 step, one stream.
source "$(dirname "$0")/../gpu_steps.sh"
for core in def wave; do
  if [ $core = wave ]; then export REDCLIFF_GEMM_CORE=wave; fi
  REDCLIFF_FORK=0 step aw_tr_$core 240 timeout -s KILL 220 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/aw/$core -o run -- python scripts/grid_step.py --replicas 128 --steps 20
  f=$(ls gpurun_out/aw/$core/*/run_kernel_trace.csv gpurun_out/aw/$core/run_kernel_trace.csv 2>/dev/null | head -n 1)
  python scripts/gemm_products.py "$f" --match k_ > gpurun_out/aw_${core}_all.txt 2>&1
  rm -f "$f"
done
