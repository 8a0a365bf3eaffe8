#!/bin/bash
# Round 5: fit_packs (concurrent packed fits) test + the packed-fit tests, the reference-grid leg with
# concurrent packs, and the k_fac_bwd_s16 stagger sweep (per-kernel times, one stream)
source "$(dirname "$0")/../gpu_steps.sh"
step e_tests 600 python -u -m pytest tests/test_gpu_pack_fit.py tests/test_gpu_replicas.py tests/test_gpu_large_pack.py -v --timeout 300 --timeout-method thread -rA
step e_refgrid 600 python bench.py --steps 5 --warmup 2 --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --no-cpu-baseline --no-north-star --no-kernel-times
step e_stagger 600 python scripts/grid_sweep.py --replicas 128 --steps 30 --rounds 2 --kernel-times --settings '[{"REDCLIFF_FORK":"0"},{"REDCLIFF_FORK":"0","REDCLIFF_S16_STAGGER":"1"},{"REDCLIFF_FORK":"0","REDCLIFF_S16_STAGGER":"2"},{"REDCLIFF_FORK":"0","REDCLIFF_S16_STAGGER":"1:odd"},{"REDCLIFF_FORK":"0","REDCLIFF_S16_STAGGER":"2:odd"},{"REDCLIFF_FORK":"0","REDCLIFF_S16_STAGGER":"1:prio"},{"REDCLIFF_FORK":"0","REDCLIFF_S16_STAGGER":"1:odd:prio"}]'
