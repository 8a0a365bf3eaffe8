#!/bin/bash
# Round 4: HIP-graph replay of the single-fit step chain vs stream launches (timing probe)
source "$(dirname "$0")/../gpu_steps.sh"
( while sleep 20; do echo "heartbeat $(date +%s)" >> gpurun_out/heartbeat.txt; done ) &
HB=$!
step f_graph_d4ic 200 python scripts/graph_probe.py --config d4ic
step f_graph_c1k4 200 python scripts/graph_probe.py --config c1k4
step f_graph_c4 200 python scripts/graph_probe.py --config c4
kill $HB
