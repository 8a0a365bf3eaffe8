#!/bin/bash
# Round 5: k_emb_tail with 4 (or 2) combine elements per thread (lib_ce4.so / lib_ce2.so): at C1(K=4) the
# tail's grid (482 workgroups at CE 4) becomes resident and replaces k_emb_combine + k_emb_final
source "$(dirname "$0")/../gpu_steps.sh"
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
  for cfg in c1k4 d4ic; do
    step z_${cfg}_base_$rep 200 $B --config $cfg
    REDCLIFF_HIP_LIB=scripts/bin/lib_ce4.so step z_${cfg}_ce4_$rep 200 $B --config $cfg
    REDCLIFF_HIP_LIB=scripts/bin/lib_ce2.so step z_${cfg}_ce2_$rep 200 $B --config $cfg
  done
done
REDCLIFF_HIP_LIB=scripts/bin/lib_ce4.so step z_tests 300 python -u -m pytest tests/test_gpu_forked.py -v --timeout 300 --timeout-method thread -rA
