#!/bin/bash
# Round 5: the embedder backward's window blocking (rc_emb_wpb / rc_emb_nbw: several integer divisions
# per workgroup) and the forward's slices per window computed by the host; the combine kernel's
# prologue 997 -> 515 instructions.  Bitwise whole fits against the previous build, single-fit steps,
# phase traces, the whole GPU suite.
source "$(dirname "$0")/../gpu_steps.sh"
P=scripts/bin/lib_prev_r5h.so
COMPARE_FITS_CFGS=c4,c1k4,d4ic,c5 COMPARE_FITS_R=1 REDCLIFF_HIP_LIB=$P step ah_dump_prev 300 python scripts/compare_fits.py dump gpurun_out/fprev_1.npz
COMPARE_FITS_CFGS=c4,c1k4,d4ic,c5 COMPARE_FITS_R=1 step ah_dump_cur 300 python scripts/compare_fits.py dump gpurun_out/fcur_1.npz
step ah_cmp 60 python scripts/compare_fits.py compare gpurun_out/fprev_1.npz gpurun_out/fcur_1.npz
rm -f gpurun_out/fprev_*.npz gpurun_out/fcur_*.npz
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
for cfg in c1k4 c4 d4ic; do
  REDCLIFF_HIP_LIB=$P step ah_prev_${cfg}_$rep 200 $B --config $cfg
  step ah_cur_${cfg}_$rep 200 $B --config $cfg
done
done
step ah_trace_c1k4 200 python scripts/phase_trace.py --config c1k4
step ah_trace_c4 200 python scripts/phase_trace.py --config c4
step ah_suite 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x
