#!/bin/bash
# Round 4: new defaults (forked packs, ept 8) against the old ones, interleaved on one box
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
S='[{}, {"REDCLIFF_FORK": "0", "REDCLIFF_EMB_FINAL_EPT": "4"}]'
step v_sweep 300 python -u scripts/grid_sweep.py --replicas 128 --steps 40 --rounds 4 --settings "$S"
step v_pf_new1 300 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40
step v_pf_old1 300 env REDCLIFF_FORK=0 REDCLIFF_EMB_FINAL_EPT=4 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40
step v_pf_new2 300 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40
step v_pf_old2 300 env REDCLIFF_FORK=0 REDCLIFF_EMB_FINAL_EPT=4 python -u scripts/pack_fit_profile.py --replicas 128 --epochs 40
kill $HB
