#!/bin/bash
# Round 5: short-latency staging in two one-workgroup chains, same bits:
#  - k_emb_bwd node staging: all factor-side dL/dw partial rounds' loads in flight together (p <= 16, K > 4)
#  - k_emb_final adjacency workgroup: the dS record sums with eight loads in flight, the p x p products'
#    operand reads and read-modify-writes batched
# (1) bitwise whole packed fits against the previous build (c4 has K = 9, n = 3); (2) single-fit steps,
# previous vs current; (3) phase traces c1k4 / c4; (4) the tests that run these kernels
source "$(dirname "$0")/../gpu_steps.sh"
P=scripts/bin/lib_prev_r5c.so
for R in 1 4; do
  COMPARE_FITS_CFGS=c4,c1k4,d4ic COMPARE_FITS_R=$R REDCLIFF_HIP_LIB=$P step ac_dump_prev_$R 300 python scripts/compare_fits.py dump gpurun_out/fprev_$R.npz
  COMPARE_FITS_CFGS=c4,c1k4,d4ic COMPARE_FITS_R=$R step ac_dump_cur_$R 300 python scripts/compare_fits.py dump gpurun_out/fcur_$R.npz
  step ac_cmp_$R 60 python scripts/compare_fits.py compare gpurun_out/fprev_$R.npz gpurun_out/fcur_$R.npz
done
rm -f gpurun_out/fprev_*.npz gpurun_out/fcur_*.npz
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
for cfg in c1k4 c4 d4ic; do
  REDCLIFF_HIP_LIB=$P step ac_prev_${cfg}_$rep 200 $B --config $cfg
  step ac_cur_${cfg}_$rep 200 $B --config $cfg
done
done
step ac_trace_c1k4 200 python scripts/phase_trace.py --config c1k4
step ac_trace_c4 200 python scripts/phase_trace.py --config c4
step ac_tests 600 python -u -m pytest tests/test_gpu_forked.py tests/test_gpu_fit_golden.py tests/test_gpu_replicas.py -v --timeout 300 --timeout-method thread -rA
