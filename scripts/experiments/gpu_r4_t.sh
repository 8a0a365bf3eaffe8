#!/bin/bash
# Round 4: two-stream (forked) packed step vs one stream across R, with the k_emb_final shape
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
S='[{"REDCLIFF_FORK": "0"}, {"REDCLIFF_FORK": "1"}, {"REDCLIFF_FORK": "0", "REDCLIFF_EMB_FINAL_EPT": "8"}, {"REDCLIFF_FORK": "1", "REDCLIFF_EMB_FINAL_EPT": "8"}, {"REDCLIFF_FORK": "1", "REDCLIFF_EMB_FINAL_EPT": "8", "REDCLIFF_GEMM_TILE": "32"}]'
for R in 128 64 32 8; do
step t_sweep_r$R 300 python -u scripts/grid_sweep.py --replicas $R --steps 40 --rounds 3 --settings "$S"
done
step t_pf_fork 300 env REDCLIFF_FORK=1 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40
step t_pf_nofork 300 env REDCLIFF_FORK=0 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40
kill $HB
