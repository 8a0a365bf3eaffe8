#!/bin/bash
# Round 6: the GPU suite on the committed tree, then the TST pack's embedder products on the other
# GEMM forms (one product per launch; the LDS-tiled matrix-core core) against the default wave-core pairs.
source "$(dirname "$0")/../gpu_steps.sh"
step dd_suite 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf
GR="--no-cpu-baseline --steps 20 --warmup 5 --replicas 128 --grid-steps 100 --fit-replicas 0 --ref-grid-epochs 0 --dp-leg-batch 0 --no-north-star --c5-steps 0 --config c4"
step dd_tst_default 300 python bench.py $GR
REDCLIFF_GEMM_SET=0 step dd_tst_set0 300 python bench.py $GR
REDCLIFF_GEMM_CORE=mfma step dd_tst_mfma 300 python bench.py $GR
step dd_tst_default2 300 python bench.py $GR
