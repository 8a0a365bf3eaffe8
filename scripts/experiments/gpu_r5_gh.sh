#!/bin/bash
# Round 5: r5g (full GPU suite, smoke, bench line) then r5h (embedder-forward windows per workgroup sweep,
# kernel times of C1(K=4) / TST, SQ counters of k_fac_bwd_s16, every 8-GPU share of the reference grids)
bash "$(dirname "$0")/gpu_r5_g.sh" && bash "$(dirname "$0")/gpu_r5_h.sh"
