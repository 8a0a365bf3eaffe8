# rocprofv3 counter passes (one counter group per run) over the single-fit D4IC bench, plus the
# kernel-trace summary of the same command; bench.py's roofline.traffic reads the FETCH/WRITE passes.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python bench.py --no-cpu-baseline --no-kernel-times --steps 50 --warmup 5 --replicas 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- $B > gpurun_out/pmc1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- $B > gpurun_out/pmc2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_sq -o run -- $B > gpurun_out/pmc3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d gpurun_out/pmc_ic -o run -- $B > gpurun_out/pmc4.log 2>&1
