#!/bin/bash
# Round 5: the pack-vs-solo history difference of the synthetic shape classes (2, 3) / (1, 12) on the
# packed-grid kernels, entry by entry in the test's order; the HipAdam vanilla test; the reference-grid
# shares with FLOP-weighted class-aware sharding
source "$(dirname "$0")/../gpu_steps.sh"
REDCLIFF_FAC_PATH=mfma REDCLIFF_EMB_PATH=gemm step j_hist_mg 300 python -u scripts/determinism_probe.py --shapes 2x3,1x12,1x3 --hist
REDCLIFF_FAC_PATH=mfma REDCLIFF_EMB_PATH=fused step j_hist_mf 300 python -u scripts/determinism_probe.py --shapes 2x3,1x12 --hist
REDCLIFF_FAC_PATH=vector REDCLIFF_EMB_PATH=gemm step j_hist_vg 300 python -u scripts/determinism_probe.py --shapes 2x3,1x12 --hist
step j_adam 300 python -u -m pytest tests/test_gpu_generic.py -k hip_adam -v --timeout 300 --timeout-method thread -rA
for sh in 0 3 5 6 7; do
  step j_share_$sh 300 python bench.py --steps 5 --warmup 2 --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --no-cpu-baseline --no-north-star --no-kernel-times --ref-grid-epochs 4 --ref-grid-share $sh
done
