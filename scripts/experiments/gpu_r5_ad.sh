#!/bin/bash
# Round 5: more single-workgroup latency, same bits: the node staging's BatchNorm operands requested
# with the staging (stored after it); the forward's last arriver loads its slice partials together;
# k_emb_final<16>'s dS batch sized to its staging width (no scratch).
# (1) bitwise whole packed fits against the previous build (c5: p = 64, the 16-element adjacency
# workgroup); (2) single-fit steps, previous vs current; (3) phase traces; (4) the tests of these kernels
source "$(dirname "$0")/../gpu_steps.sh"
P=scripts/bin/lib_prev_r5d.so
for R in 1 4; do
  COMPARE_FITS_CFGS=c4,c1k4,d4ic,c5 COMPARE_FITS_R=$R REDCLIFF_HIP_LIB=$P step ad_dump_prev_$R 300 python scripts/compare_fits.py dump gpurun_out/fprev_$R.npz
  COMPARE_FITS_CFGS=c4,c1k4,d4ic,c5 COMPARE_FITS_R=$R step ad_dump_cur_$R 300 python scripts/compare_fits.py dump gpurun_out/fcur_$R.npz
  step ad_cmp_$R 60 python scripts/compare_fits.py compare gpurun_out/fprev_$R.npz gpurun_out/fcur_$R.npz
done
rm -f gpurun_out/fprev_*.npz gpurun_out/fcur_*.npz
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
for cfg in c1k4 c4 d4ic; do
  REDCLIFF_HIP_LIB=$P step ad_prev_${cfg}_$rep 200 $B --config $cfg
  step ad_cur_${cfg}_$rep 200 $B --config $cfg
done
done
step ad_trace_c1k4 200 python scripts/phase_trace.py --config c1k4
step ad_trace_c4 200 python scripts/phase_trace.py --config c4
step ad_tests 600 python -u -m pytest tests/test_gpu_forked.py tests/test_gpu_fit_golden.py tests/test_gpu_replicas.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -rA
