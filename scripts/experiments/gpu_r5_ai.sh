#!/bin/bash
# Round 5 (against the r5af build: includes r5ah's host window blocking): the adjacency workgroup's p x p products (one wave, instruction-issue bound): half the
# epilogue for p <= 16 (rows 16..31 of the 32x32 tile are padding), the supports' dense copy out by
# every thread, the supports' divider from the host.  Bitwise whole fits (R = 1 and 4), single-fit
# steps, phase traces, the instruction-fetch experiment, the whole GPU suite.
source "$(dirname "$0")/../gpu_steps.sh"
P=scripts/bin/lib_prev_r5h.so
COMPARE_FITS_CFGS=c4,c1k4,d4ic,c5 COMPARE_FITS_R=1 REDCLIFF_HIP_LIB=$P step ai_dump_prev 300 python scripts/compare_fits.py dump gpurun_out/fprev_1.npz
COMPARE_FITS_CFGS=c4,c1k4,d4ic,c5 COMPARE_FITS_R=1 step ai_dump_cur 300 python scripts/compare_fits.py dump gpurun_out/fcur_1.npz
step ai_cmp 60 python scripts/compare_fits.py compare gpurun_out/fprev_1.npz gpurun_out/fcur_1.npz
rm -f gpurun_out/fprev_*.npz gpurun_out/fcur_*.npz
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
for cfg in c1k4 c4 d4ic; do
  REDCLIFF_HIP_LIB=$P step ai_prev_${cfg}_$rep 200 $B --config $cfg
  step ai_cur_${cfg}_$rep 200 $B --config $cfg
done
done
step ai_trace_c1k4 200 python scripts/phase_trace.py --config c1k4
step ai_trace_c4 200 python scripts/phase_trace.py --config c4
COMPARE_FITS_CFGS=c4,c1k4 COMPARE_FITS_R=4 REDCLIFF_HIP_LIB=$P step ai_dump_prev4 300 python scripts/compare_fits.py dump gpurun_out/fprev_4.npz
COMPARE_FITS_CFGS=c4,c1k4 COMPARE_FITS_R=4 step ai_dump_cur4 300 python scripts/compare_fits.py dump gpurun_out/fcur_4.npz
step ai_cmp4 60 python scripts/compare_fits.py compare gpurun_out/fprev_4.npz gpurun_out/fcur_4.npz
rm -f gpurun_out/fprev_*.npz gpurun_out/fcur_*.npz
step ai_suite 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x
