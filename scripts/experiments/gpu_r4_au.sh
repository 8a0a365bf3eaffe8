#!/bin/bash
# Round 4: HIP graph of the forked C1(K=4) / TST single-fit step chain vs stream launches (timing probe)
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step au_c1k4 200 python -u scripts/graph_probe.py --config c1k4 --steps 20
step au_c4 200 python -u scripts/graph_probe.py --config c4 --steps 20
step au_d4ic 200 python -u scripts/graph_probe.py --config d4ic --steps 20
kill $HB
