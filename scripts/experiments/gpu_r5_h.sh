#!/bin/bash
# Round 5: windows per embedder-forward workgroup (REDCLIFF_EMB_SB, read once per process) on the single
# fits C1(K=4) (north star), TST and D4IC; SQ counters of the R = 128 grid step (k_fac_bwd_s16)
source "$(dirname "$0")/../gpu_steps.sh"
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
for cfg in c1k4 c4 d4ic; do
  for sb in 1 2 4; do
    REDCLIFF_EMB_SB=$sb step h_sb_${cfg}_${sb}_$rep 200 $B --config $cfg
  done
done
done
step h_sq 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --kernel-include-regex k_fac_bwd_s16 --output-format csv -d gpurun_out/h/sq -o run -- python scripts/grid_step.py --replicas 128 --steps 3
for sh in 0 1 2 3 4 5 6 7; do
  step h_share_$sh 300 python bench.py --steps 5 --warmup 2 --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --no-cpu-baseline --no-north-star --no-kernel-times --ref-grid-epochs 4 --ref-grid-share $sh
done
step h_kt_c1k4 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --config c1k4
step h_kt_c4 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --config c4
