#!/bin/bash
# Round 5: (1) fork / join event scope (REDCLIFF_EVENT_SCOPE) on the single fits C1(K=4) / TST with the
# channel-sliced embedder forward (default 300 columns); (2) k_fac_bwd_s16 at 3 waves per SIMD
# (scripts/bin/lib_s16w3.so, -DRC_S16_BWD_WAVES=3): R = 128 grid kernel times and bitwise packed fits
source "$(dirname "$0")/../gpu_steps.sh"
W=scripts/bin/lib_s16w3.so
B="python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-north-star --replicas 1 --fit-replicas 0 --dp-leg-batch 0 --ref-grid-epochs 0 --no-kernel-times"
for rep in 1 2; do
  for cfg in c1k4 c4; do
    step m_${cfg}_base_$rep 200 $B --config $cfg
    REDCLIFF_EVENT_SCOPE=device step m_${cfg}_device_$rep 200 $B --config $cfg
    REDCLIFF_EVENT_SCOPE=nofence step m_${cfg}_nofence_$rep 200 $B --config $cfg
  done
done
step m_sweep_cur 300 python scripts/grid_sweep.py --replicas 128 --steps 30 --rounds 2 --kernel-times --settings '[{"REDCLIFF_FORK":"0"}]'
REDCLIFF_HIP_LIB=$W step m_sweep_w3 300 python scripts/grid_sweep.py --replicas 128 --steps 30 --rounds 2 --kernel-times --settings '[{"REDCLIFF_FORK":"0"}]'
step m_sweep_cur2 300 python scripts/grid_sweep.py --replicas 128 --steps 30 --rounds 2 --kernel-times --settings '[{"REDCLIFF_FORK":"0"}]'
REDCLIFF_HIP_LIB=$W step m_sweep_w3_2 300 python scripts/grid_sweep.py --replicas 128 --steps 30 --rounds 2 --kernel-times --settings '[{"REDCLIFF_FORK":"0"}]'
COMPARE_FITS_R=32 step m_dump_cur 300 python scripts/compare_fits.py dump gpurun_out/mcur.npz
COMPARE_FITS_R=32 REDCLIFF_HIP_LIB=$W step m_dump_w3 300 python scripts/compare_fits.py dump gpurun_out/mw3.npz
step m_cmp 60 python scripts/compare_fits.py compare gpurun_out/mcur.npz gpurun_out/mw3.npz
rm -f gpurun_out/mcur.npz gpurun_out/mw3.npz
