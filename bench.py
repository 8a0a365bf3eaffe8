#!/usr/bin/env python
"""REDCLIFF-S cMLP factor-model fitting on MI355X: fused fwd+bwd windows/sec.

A "step" is one REDCLIFF-S batch_update in the combined training phase (embedder +
K x p factor networks forward, conditional-GC penalties, backward, Adam on both
optimizer groups) over one batch of B=128 synthetic windows resident in HBM.
Default workload = BASELINE.json configs[1]: REDCLIFF-S w/ state smoothing, D4IC-shaped
(p=10 channels, gen_lag 4, 4 factors, hidden 100, DGCNN F=20 / 2 layers / 30 hidden,
windows of 21 steps, labels (N, K, 1)); D4IC itself is not in the image, so the windows
are synthetic with the same shapes.

    python bench.py [--gpus N --steps K --warmup W] [--mode fit|dp]

--gpus N > 1 without a torch.distributed launcher: this process starts N ranks itself
(torch.distributed.run, 127.0.0.1) before touching the GPU and exits with their status.

mode "fit" (default): every rank runs an independent fit (grid-search replicas shard one per
GPU, no collective); value = all windows processed / max-over-ranks time ("scaling": "weak").
The same line carries the packed grid search (R fits per launch, windows/s and fits/hour)
and, at N = 1, the north-star ratio config (10 channels / 5 lags / 4 factors) with its own
CPU baseline.
mode "dp": BASELINE configs[3] -- one TST-shaped fit data-parallel over the N ranks (shards of
every global batch, one RCCL all-reduce of the flat gradient per update).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))

FP32_PEAK_TFLOPS = 157.3  # MI355X dense FP32 (vector == f32 MFMA rate), MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0
METRIC = "cMLP-factor fwd+bwd windows/sec/GPU; grid-search fits/hour on 8 GPUs"

CONFIGS = {
    # BASELINE.json configs[1]: D4IC-shaped, 4 factors (train/REDCLIFF_S_CMLP_Smooth_d4IC_BSCgs4ParsimSmo0_cached_args.txt)
    "d4ic": dict(p=10, L=4, K=4, nsup=4, h=100, F=20, n=2, H=30, B=128, T=21, label_T=1, lrA=2e-4, lrB=5e-4,
                 workload="REDCLIFF-S cMLP w/ state smoothing, D4IC-shaped (p=10, gen_lag=4, K=4, h=100, "
                          "DGCNN F=20/2 layers/30 hidden), combined-phase batch_update, B=128"),
    # north-star ratio config: 10 channels / 5 lags / 4 factors (synthetic sVAR shapes)
    "c1k4": dict(p=10, L=5, K=4, nsup=4, h=25, F=16, n=3, H=100, B=128, T=100, label_T=100, lrA=5e-4, lrB=5e-4,
                 workload="REDCLIFF-S cMLP w/ state smoothing, synthetic sVAR (p=10, gen_lag=5, K=4, h=25, "
                          "DGCNN F=16/3 layers/100 hidden), combined-phase batch_update, B=128"),
    # BASELINE.json configs[3]: TST-shaped (region averages), data-parallel
    "c4": dict(p=12, L=4, K=9, nsup=3, h=25, F=16, n=3, H=100, B=128, T=150, label_T=150, lrA=5e-4, lrB=5e-4,
               workload="REDCLIFF-S TST-shaped (p=12, gen_lag=4, K=9, nsup=3, h=25, DGCNN 16/3/100), B=128"),
    # BASELINE.json configs[4]: scaled synthetic stress (large grouped contraction)
    "c5": dict(p=64, L=20, K=8, nsup=8, h=25, F=64, n=3, H=100, B=128, T=128, label_T=128, lrA=5e-4, lrB=5e-4,
               workload="REDCLIFF-S stress (p=64, gen_lag=20, K=8, h=25, DGCNN F=64/3 layers/100 hidden), B=128"),
}


def flops_per_window(c):
    """Algorithmic FLOPs per window: useful work only (the reference's 3x
    embedder re-evaluation is not counted)."""
    p, L, K, h, F, n, H = c["p"], c["L"], c["K"], c["h"], c["F"], c["n"], c["H"]
    fac_fwd = 2 * K * p * h * (p * L + 1)
    fac_bwd = 2 * K * p * h * (p * L + 2)
    emb_fwd = 2 * ((n - 1) * p * p * F + n * p * F * H + 64 * p * H + 64 * K) + 4 * p * F
    emb_bwd = 2 * emb_fwd
    pen = 6 * K * p * p * min(L, F) + 6 * K * p * p + K * (K - 1) * p * p
    return dict(fac_fwd=fac_fwd, fac_bwd=fac_bwd + pen, emb_fwd=emb_fwd, emb_bwd=emb_bwd, emb_final=0, pen=pen,
                total=fac_fwd + fac_bwd + emb_fwd + emb_bwd + pen)


def short_factor_kernels(c):
    """The matrix-core factor path runs the 16-unit short-contraction kernels (k_fac_*_s16) when
    p*L <= 64 (rc_factor_mfma.hip rc_fac_short; REDCLIFF_FAC_SHORT=0 selects the 32-unit ones)."""
    return c["p"] * c["L"] <= 64 and os.environ.get("REDCLIFF_FAC_SHORT") != "0"


def roofline_of(ktimes, fl, windows_per_launch, traffic_cfg, short=False, chains=()):
    """Roofline object of the dominant kernel: algorithmic FLOPs per launch (SURVEY 8(d)
    per-window counts x the windows one launch processes) / its average HIP-event duration.
    Timing slots: "emb_fwd" = k_forward (embedder + vector-path factor forward in one launch)
    or the GEMM embedder's forward chain; on the matrix-core path "fac_fwd" = k_xwin +
    k_fac_fwd_mfma, "fac_mix" = k_fac_mix, "fac_bwd" = k_fac_bwd_mfma.  With two kernel chains
    on two streams the slots overlap in time (the step is shorter than their sum)."""
    fl = dict(fl)
    mfma = ktimes.get("fac_mix", (0, 0))[1] > 0
    merged = False
    if mfma:  # k_fac_mix carries the penalty terms, k_fac_bwd_mfma the dW0 contraction
        fl["fac_mix"] = fl["pen"]
        fl["fac_bwd"] -= fl["pen"]
    elif ktimes.get("fac_fwd", (0, 0))[1] == 0:
        fl["emb_fwd"] += fl["fac_fwd"]
        if ktimes.get("fac_bwd", (0, 0))[1] == 0 and ktimes.get("emb_bwd", (0, 0))[1] > 0:
            # k_bwd_merged: the factor and embedder backward in one launch (emb_bwd slot)
            merged = True
            fl["emb_bwd"] += fl["fac_bwd"]
    # chains: timing slots that hold a chain of launches (the GEMM-shaped embedder's products), not
    # one kernel -- reported, but not candidates for the dominant KERNEL
    dom = max((k for k in ktimes if k in fl and k != "supports" and k not in chains), key=lambda k: ktimes[k][0])
    avg_ms = ktimes[dom][0]
    flops = fl.get(dom, 0) * windows_per_launch
    achieved = flops / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    kname = {"emb_fwd": "k_forward", "fac_fwd": "k_fac_fwd_s16" if short else "k_fac_fwd_mfma",
             "fac_bwd": ("k_fac_bwd_s16" if short else "k_fac_bwd_mfma") if mfma else "k_fac_bwd",
             "emb_bwd": "k_bwd_merged" if merged else "k_emb_bwd", "emb_final": "k_emb_final",
             "fac_mix": "k_fac_mix"}[dom]
    return {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 4), "peak": FP32_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / FP32_PEAK_TFLOPS, 6),
            "traffic": pmc_traffic(kname, traffic_cfg) if traffic_cfg else None,
            "avg_launch_us": round(avg_ms * 1e3, 2),
            "algorithmic_flops_per_launch": flops,
            "kernel_avg_us": dict((k, round(v[0] * 1e3, 2)) for k, v in ktimes.items())}


def synth(c, N, seed):
    rng = np.random.RandomState(seed)
    X = rng.randn(N, c["T"], c["p"]).astype(np.float32)
    for t in range(2, c["T"]):
        X[:, t] += 0.4 * X[:, t - 1] - 0.2 * X[:, t - 2]
    X /= X.std()
    if c["label_T"] == 1:
        Y = np.zeros((N, c["K"], 1), np.float32)
        Y[np.arange(N), rng.randint(0, c["K"], N), 0] = 10.0
    else:
        Y = np.zeros((N, c["K"], c["label_T"]), np.float32)
        Y[np.arange(N), rng.randint(0, c["K"], N), :] = 1.0
    return torch.from_numpy(X), torch.from_numpy(Y)


def coeffs(K, p, forecast=10.0, adj=0.1):
    denom = sum(float(i) for i in range(1, K)) if K > 1 else 1.0
    return {"FORECAST_COEFF": forecast, "FACTOR_SCORE_COEFF": 100.0, "FACTOR_COS_SIM_COEFF": 1.0 / denom,
            "FACTOR_WEIGHT_L1_COEFF": 1e-3, "FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF": 0.0,
            "ADJ_L1_REG_COEFF": adj / K / np.sqrt(p * p - 1.0), "DAGNESS_REG_COEFF": 0.0,
            "DAGNESS_LAG_COEFF": 0.0, "DAGNESS_NODE_COEFF": 0.0}


def build_model(cls, c, seed, pre=1, acc=1, **cw):
    K, p = c["K"], c["p"]
    eargs = [("num_features_per_node", c["F"]), ("num_graph_conv_layers", c["n"]), ("num_hidden_nodes", c["H"]),
             ("sigmoid_eccentricity_coeff", 10.0)]
    torch.manual_seed(seed)
    return cls(p, c["L"], [c["h"]], c["F"], [0], c["L"], 1, K, c["nsup"], coeffs(K, p, **cw), False, "DGCNN", eargs,
               "conditional_factor_fixed_embedder", "apply_factor_weights_after_sim_completion", num_sims=1,
               training_mode="pretrain_embedder_then_acclimate_factors_then_combined", num_pretrain_epochs=pre,
               num_acclimation_epochs=acc)


def adam_pair(m, c):
    oA = torch.optim.Adam(m.gen_model[0].parameters(), lr=c["lrA"], betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    oB = torch.optim.Adam(m.gen_model[1].parameters(), lr=c["lrB"], betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    return oA, oB


def host_cores():
    """CPUs this process may actually run on: the affinity mask, capped by a cgroup CPU quota
    when one is set (cgroup v2 cpu.max / v1 cfs_quota) -- os.cpu_count() reports the whole
    machine even where a job gets a share of it."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = float(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = float(f.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is not None:
        n = min(n, max(1, int(np.ceil(quota))))
    return int(os.environ.get("REDCLIFF_CPU_THREADS", n))


def _oracle_rate(c, threads, seconds):
    """Combined-phase batch_updates of the oracle on `threads` threads for ~`seconds`:
    (steps, elapsed seconds)."""
    from oracle.redcliff_oracle import OracleREDCLIFF
    torch.set_num_threads(threads)
    m = build_model(OracleREDCLIFF, c, seed=0)
    oA, oB = adam_pair(m, c)
    X, Y = synth(c, 4 * c["B"], seed=1)
    bs = [(X[i:i + c["B"]], Y[i:i + c["B"]]) for i in range(0, X.shape[0], c["B"])]
    m.batch_update(2, 0, bs[0][0], bs[0][1], oA, oB, 1)  # warm-up (combined phase)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        Xb, Yb = bs[n % len(bs)]
        m.batch_update(2, n, Xb, Yb, oA, oB, 1)
        n += 1
    return n, time.perf_counter() - t0


def cpu_baseline(c, seconds):
    """The oracle (CPU restatement keeping the reference's op structure) on the host cores, at
    1 / 8 / 16 / all threads (the best rate is the baseline; all rates are reported)."""
    cores = host_cores()
    counts = sorted(set(t for t in (1, 8, 16, cores) if t <= cores))
    prev = torch.get_num_threads()
    rates = {}
    try:
        for t in counts:
            n, dt = _oracle_rate(c, t, seconds / len(counts))
            rates[t] = (n * c["B"] / dt, n, dt)
    finally:
        torch.set_num_threads(prev)
    best = max(rates, key=lambda t: rates[t][0])
    v, n, dt = rates[best]
    return {"value": round(v, 2), "unit": "windows/s", "cores": best, "host_cpu_count": os.cpu_count(),
            "host_cores_available": cores, "kind": "port",
            "by_threads": dict((str(t), round(r[0], 2)) for t, r in rates.items()),
            "sample": "%d combined-phase batch_updates of B=%d (%.1f s) with oracle/redcliff_oracle.py (reference op "
                      "structure: per-sample loops, autograd, torch.optim.Adam); best of %s threads = %d "
                      "(%d CPUs available to this job; os.cpu_count() = %s)"
                      % (n, c["B"], dt, "/".join(str(t) for t in counts), best, cores, os.cpu_count())}


def _cpu_fit_worker(c, seconds, q):
    torch.set_num_threads(1)
    n, dt = _oracle_rate(c, 1, seconds)
    q.put((n, dt))


def cpu_fits_per_hour(c, seconds, steps_per_fit):
    """The reference's CPU grid search: one fit per core, each single-threaded
    (torch.set_num_threads(1)).  P concurrent one-thread oracle processes (P =
    the CPUs available to this job) run combined-phase batch_updates for ~`seconds`; the
    aggregate step rate over all of them gives fits/hour (training steps only).  At most 15
    workers: the GPU box admits 16 processes with the card open, this one included, and a
    spawned interpreter that imports torch counts even with the devices hidden from it."""
    import multiprocessing as mp
    P = min(host_cores(), int(os.environ.get("REDCLIFF_CPU_FIT_PROCS", 15)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_cpu_fit_worker, args=(c, seconds, q)) for _ in range(P)]
    hide = ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES")
    saved = dict((k, os.environ.get(k)) for k in hide)
    try:
        for k in hide[:2]:
            os.environ[k] = ""  # the workers are CPU-only: inherited at spawn
        for pr in procs:
            pr.start()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    res = [q.get(timeout=600) for _ in procs]
    for pr in procs:
        pr.join(timeout=60)
    steps = sum(n for n, _ in res)
    wall = max(dt for _, dt in res)
    rate = steps / wall  # aggregate steps per second over the P processes
    return {"value": round(rate * 3600.0 / steps_per_fit, 2), "unit": "fits/hour", "cores": P,
            "host_cpu_count": os.cpu_count(), "kind": "port",
            "host_cores_available": host_cores(),
            "sample": "%d concurrent single-thread oracle processes (one fit per core, the reference's grid), "
                      "%d combined-phase batch_updates of B=%d in %.1f s in all (%.3f s per step per process) x %d "
                      "training steps per fit; validation and GC tracking NOT counted, so this over-states the CPU "
                      "rate" % (P, steps, c["B"], wall, P * wall / max(steps, 1), steps_per_fit)}


def hbm_roofline(c, eng, ms_per_step, ktimes_roof):
    """HBM side of the roofline: algorithmic bytes of one step -- the windows,
    4 (Lmax p + p + K) B each, plus 36 B per parameter (read W in forward and backward, write
    the gradient, read and write both Adam moments, write W) -- over the step time; and the
    dominant kernel's measured HBM bytes (PMC) over its launch time."""
    P = int(eng.emb.numel() + eng.fac.numel())
    Lmax = c["T"] - 1
    step_bytes = c["B"] * 4 * (Lmax * c["p"] + c["p"] + c["K"]) + 36 * P
    ach = step_bytes / (ms_per_step * 1e-3) / 1e9
    out = {"bound": "hbm", "scope": "whole step", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(ach / HBM_PEAK_GBS, 6), "algorithmic_bytes_per_step": step_bytes, "params": P}
    if ktimes_roof and ktimes_roof.get("traffic"):
        t = ktimes_roof["traffic"]
        out["dominant_kernel"] = {"kernel": ktimes_roof["kernel"], "measured_bytes": round(t),
                                  "achieved": round(t / (ktimes_roof["avg_launch_us"] * 1e-6) / 1e9, 2),
                                  "frac": round(t / (ktimes_roof["avg_launch_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 6)}
    return out


def pmc_traffic(kernel_name, cfg):
    """HBM bytes per launch of ``kernel_name`` from the committed rocprofv3 PMC passes, condensed by
    scripts/pmc_traffic.py into profiles/pmc_traffic.json: FETCH_SIZE x 2 (gfx950 under-count,
    MI355X_MICROARCH.md HBM) + WRITE_SIZE.  cfg "<config>" takes the launches with the SMALLEST grid (the
    single fit); "<config>_r<R>" (a packed grid search) the LARGEST grid (the R-replica launches); the
    newest round that measured the kernel at that config first (kernels change between rounds)."""
    base, packed = (cfg.rsplit("_r", 1)[0], True) if "_r" in cfg else (cfg, False)
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        recs = [r for r in json.load(f) if r["config"] == base and r["kernel"] == kernel_name]
    if not recs:
        return None
    rnd = max(r["round"] for r in recs)
    recs = [r for r in recs if r["round"] == rnd]
    pick = (max if packed else min)(recs, key=lambda r: r["grid_size"])
    return (2.0 * pick["fetch_kib"] + pick["write_kib"]) * 1024.0  # counters are in KiB


# --------------------------------------------------------------------------- timing helpers
def timed(fn, dist, dev):
    """fn() bracketed by barrier + synchronize on both sides; max over ranks.  A one-rank group
    has nobody to wait for: its barrier (an RCCL launch and a host round trip, ~2 us per step of a
    20-step region, profiles/r04_steady_state_a.log) is skipped."""
    if dist is not None and dist.get_world_size() == 1:
        dist = None
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        # the coordination group of --mode fit is gloo (host tensors); --mode dp's is RCCL
        on_host = dist.get_backend() == "gloo"
        t = torch.tensor([el], device=None if on_host else dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def preheat(plan, start, seconds):
    """Untimed steps, after the W warm-up steps, until the device has been busy for `seconds`: a
    GPU that idled through the host-side setup runs its first timed region ~7 % slower than the
    next one (clock ramp; profiles/r04_steady_state_a.log: 20-step regions 0.0651 -> 0.0610 ->
    0.0605 ms per step, 300 steps 0.0586).  Returns the number of extra steps."""
    if seconds <= 0:
        return 0
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        plan(20, start + n).run()
        torch.cuda.synchronize()
        n += 20
    return n


def single_fit(c, args, dev, rank, nbatch=32):
    """One independent fit: model, optimizers, device-resident batches; returns the engine,
    a plan factory for n steps starting at batch `start` (built outside any timed region)."""
    import redcliff_amd
    B = c["B"]
    model = build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=rank).to(dev)
    oA, oB = adam_pair(model, c)
    X, Y = synth(c, nbatch * B, seed=100 + rank)
    eng = model.engine()
    ds = eng.cache_dataset([(X[i:i + B], Y[i:i + B]) for i in range(0, X.shape[0], B)])
    d = eng.workspace(ds["Bmax"], ds["T"])

    def plan(nsteps, start):
        idx = (np.arange(nsteps) + start) % nbatch
        stats = ds["stats"][torch.as_tensor(idx, device=dev)].contiguous()
        return eng.plan_steps("combined", ds["X"], ds["lab"], stats, d, ds["rows"][idx], ds["sizes"][idx], oA, oB)

    return eng, plan


def kernel_times_of(run):
    from redcliff_amd import _native as nat
    nat.kernel_timing(True)
    run()
    torch.cuda.synchronize()
    kt = nat.kernel_times()
    nat.kernel_timing(False)
    return dict((k, (ms / n if n else 0.0, n)) for k, (ms, n) in kt.items())


def run_grid(c, args, dev, rank, dist):
    """Time args.grid_steps combined-phase steps of R packed grid-search replicas."""
    import redcliff_amd
    K, p = c["K"], c["p"]
    R = args.replicas
    models, opts = [], []
    for i in range(R):
        m = build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=1000 * rank + i,
                        forecast=(10.0, 1.0)[i % 2], adj=(0.1, 0.01)[(i // 2) % 2]).to(dev)
        # vary what the reference grid varies (train/...gsSmooth1.py:278-309): lrs and coefficients
        cc = dict(c, lrA=(5e-4, 1e-4)[(i // 4) % 2], lrB=(5e-4, 1e-4)[(i // 8) % 2])
        models.append(m)
        opts.append(adam_pair(m, cc))
    pack = redcliff_amd.ReplicaPack(models, opts)
    nbatch = 8
    X, Y = synth(c, nbatch * c["B"], seed=200 + rank)
    ds = pack.cache_dataset([(X[i:i + c["B"]], Y[i:i + c["B"]]) for i in range(0, X.shape[0], c["B"])])

    def steps(n, start):
        idx = (np.arange(n) + start) % nbatch
        st = ds["stats"][torch.as_tensor(idx, device=dev)].contiguous()
        return lambda: pack.run_steps(["combined"], ds, ds["rows"][idx], ds["sizes"][idx], st)

    steps(5, 0)()
    extra = 0  # untimed steps until the device has been busy for args.preheat_s (as the single fit)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < getattr(args, "preheat_s", 0.0):
        steps(20, 5 + extra)()
        torch.cuda.synchronize()
        extra += 20
    el = timed(steps(args.grid_steps, 5 + extra), dist, dev)
    return el, R, steps


def fits_per_hour(c, args, dev, rank, dist, world):
    """Whole grid-search fits (the reference's unit of work: one SLURM task = one fit,
    train/REDCLIFF_S_CMLP_tst100hzRerun1024AvgReg_gsSmooth1.py:125-160) packed R per GPU:
    ReplicaPack.fit over a fixed-epoch schedule (pretrain, acclimation, combined epochs;
    per-epoch GC tracking, validation and best-model bookkeeping per replica)."""
    import redcliff_amd
    R, E = args.fit_replicas, args.fit_epochs
    pre, acc = max(1, E // 5), max(1, E // 10)
    ntr, nva = args.fit_train_batches, 2
    models, opts = [], []
    for i in range(R):
        m = build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=5000 * rank + i, pre=pre, acc=acc,
                        forecast=(10.0, 1.0)[i % 2], adj=(0.1, 0.01)[(i // 2) % 2]).to(dev)
        models.append(m)
        opts.append(adam_pair(m, dict(c, lrA=(5e-4, 2e-4)[(i // 4) % 2], lrB=(5e-4, 1e-4)[(i // 8) % 2])))
    X, Y = synth(c, (ntr + nva) * c["B"], seed=300 + rank)
    B = c["B"]
    train = [(X[i:i + B], Y[i:i + B]) for i in range(0, ntr * B, B)]
    val = [(X[i:i + B], Y[i:i + B]) for i in range(ntr * B, (ntr + nva) * B, B)]
    rng = np.random.RandomState(7)
    true_gc = [(rng.rand(c["p"], c["p"], c["L"]) < 0.2).astype(np.float64) for _ in range(c["K"])]
    # untimed warm-up: a 3-epoch fit of a copy of the pack (kernels loaded, the caching allocators
    # holding the pack-sized buffers), as a grid search's later packs find the process
    import copy
    wm = [copy.deepcopy(m) for m in models]
    wpack = redcliff_amd.ReplicaPack(wm, [adam_pair(m, c) for m in wm])
    wpack.fit(None, train, val, max_iter=3, lookback=10 ** 6, check_every=10 ** 6, GC=true_gc)
    del wpack, wm
    torch.cuda.synchronize()
    pack = redcliff_amd.ReplicaPack(models, opts)

    def fit():
        pack.fit(None, train, val, max_iter=E, lookback=10 ** 6, check_every=10 ** 6, GC=true_gc)

    el = timed(fit, dist, dev)
    return {"replicas_per_gpu": R, "epochs_per_fit": E, "train_windows": ntr * B, "val_windows": nva * B,
            "seconds": round(el, 3), "value": round(world * R * 3600.0 / el, 1), "unit": "fits/hour",
            "note": "fixed-epoch D4IC-shaped fits (%d pretrain, %d acclimation, %d combined epochs), early stopping "
                    "disabled so every fit does the same work; per-epoch GC tracking + validation on the GPU; "
                    "after an untimed 3-epoch warm-up fit of a copy of the pack" % (pre, acc, E - pre - acc)}


# --------------------------------------------------------------------------- the reference's grids
def tst_grid_points():
    """The TST grid (train/REDCLIFF_S_CMLP_tst100hzRerun1024AvgReg_gsSmooth1.py:278-309, 1536 points, in
    itertools.product order): per point the axes that vary -- gen_lr, FORECAST, COS_SIM, SMOOTHING,
    ADJ_L1, num_pretrain_epochs, num_acclimation_epochs, graph-conv layers, embed_lag, embed_lr."""
    import itertools
    axes = (("gen_lr", (5e-4, 1e-4)), ("forecast", (10.0, 1.0)), ("cos", (10.0, 1.0)), ("smooth", (25.0, 0.025)),
            ("adj", (0.1, 0.01)), ("pre", (100, 50)), ("acc", (15, 100)), ("layers", (2, 3)), ("lag", (16, 32, 64)),
            ("embed_lr", (5e-4, 1e-4)))
    return [dict(zip([a for a, _ in axes], v)) for v in itertools.product(*[x for _, x in axes])]


def synthetic_grid_points():
    """(K, p) of the 990 data sets of the synthetic grid in the reference driver's order
    (train/REDCLIFF_S_CMLP_synSysInnovGauss1030_BSCgsSmooth3Parsim.py:140-1131: numF / numN of each
    name; num_factors = num_supervised_factors = numF, :97-100)."""
    order = [(10, 12), (10, 6), (9, 12), (9, 6), (8, 12), (8, 6), (7, 12), (7, 6), (6, 12), (6, 6), (5, 12), (5, 6),
             (5, 3), (4, 12), (4, 6), (4, 3), (3, 12), (3, 6), (3, 3), (2, 12), (2, 6), (2, 3), (1, 12), (1, 6), (1, 3)]
    counts = {(1, 3): 30, (1, 6): 105, (1, 12): 90, (2, 3): 30, (2, 6): 90, (2, 12): 90, (3, 3): 15, (3, 6): 60,
              (3, 12): 60, (4, 3): 15, (4, 6): 45, (4, 12): 45, (5, 3): 15, (5, 6): 30, (5, 12): 45, (6, 6): 30,
              (6, 12): 30, (7, 6): 15, (7, 12): 30, (8, 6): 15, (8, 12): 30, (9, 6): 15, (9, 12): 30, (10, 6): 15,
              (10, 12): 15}
    return [kp for kp in order for _ in range(counts[kp])]


SYN_GRID_NOTE = (
    "models the synthetic grid as its data sets define it: K = nsup = the numF of the data set's name, and for "
    "K = 1 FACTOR_COS_SIM_COEFF is left undivided (no cosine pairs exist, the term is 0).  The reference driver "
    "as written does not train 255 of these 990 tasks: it reads K as int(data_set_name[4]) "
    "(train/REDCLIFF_S_CMLP_synSysInnovGauss1030_BSCgsSmooth3Parsim.py:99-100), so 'numF10' gives K = 1, and "
    "for K = 1 it divides FACTOR_COS_SIM_COEFF by sum([]) = 0 (:101-102), a ZeroDivisionError before the fit "
    "starts (the 225 numF1 tasks and the 30 numF10 tasks)")


# Time model of one GPU's share of a reference grid (a packed fit per shape class, the share's packs run
# concurrently by fit_packs): seconds ~ per_pack x packs + per_fit x fits + per_mflop x the fits' summed
# algorithmic MFLOP per window (flops_per_window).  Least-squares fit over all 16 shares of both grids
# timed one by one on one GPU (profiles/r06_refgrid_all_shares_c.json; 0.32 - 0.71 s, residuals within
# 0.04 s).  Used to pick the share a one-GPU run times beside share 0 (the slowest one by the model), and
# by the opt-in min-max cut (--ref-grid-model 1).  That cut is NOT the default: back to back on one box
# it helped the TST grid (slowest share 0.767 -> 0.733 s) and hurt the synthetic one (0.504 -> 0.563 s;
# profiles/r06_refgrid_all_shares_h_{old,model}.json) -- the same share varies by up to 10 % from run to
# run, about the model's own error, so the round-5 FLOP-weighted cut stays.
REF_GRID_COST = dict(per_pack=0.0728, per_fit=0.00065, per_mflop=0.001202)


def ref_grid_shares(cut="flop", model=REF_GRID_COST):
    """Both reference grids dealt to an 8-GPU node by class-aware sharding (redcliff_amd.shard_grid).
    cut "flop": the points cost their class's algorithmic FLOPs per window and are cut into equal-cost
    runs (min_piece 32); cut "model": each point costs per_fit + per_mflop x its MFLOP per window, each
    class a share touches per_pack, and the 8 contiguous runs minimise the largest share's modelled
    time (piece_cost).  {grid: (points, class of each point, FLOPs of each point, [point indices of share
    s for s in 0..7], [modelled seconds of share s])}."""
    from redcliff_amd import shard_grid
    out = {}
    pts = tst_grid_points()
    base = CONFIGS["c4"]
    cls = [(q["lag"], q["layers"]) for q in pts]
    fl = [flops_per_window(dict(base, F=q["lag"], n=q["layers"], T=q["lag"] + 4))["total"] for q in pts]
    kp = synthetic_grid_points()
    fl_syn = [flops_per_window(_syn_cfg(k, p))["total"] for k, p in kp]
    for name, keys, f in (("tst", cls, fl), ("synthetic", kp, fl_syn)):
        tcost = [model["per_fit"] + model["per_mflop"] * x / 1e6 for x in f]
        if cut == "flop":
            shares = [shard_grid(len(keys), 8, s, classes=keys, cost=list(f), min_piece=32) for s in range(8)]
        else:
            shares = [shard_grid(len(keys), 8, s, classes=keys, cost=tcost, piece_cost=model["per_pack"])
                      for s in range(8)]
        loads = [float(sum(tcost[i] for i in sh) + model["per_pack"] * len(set(keys[i] for i in sh))) for sh in shares]
        out[name] = (pts if name == "tst" else kp, keys, f, shares, loads)
    return out


def _syn_cfg(K, p):
    """The synthetic grid's model at (K, p) (cached args: gen_lag 4, h 25, DGCNN 16 / 3 / 100)."""
    return dict(CONFIGS["c4"], p=p, K=K, nsup=K, F=16, n=3, T=100, label_T=100)


def reference_grids(args, dev, rank, world, dist):
    """fits/hour on the reference's own grids, dealt to an 8-GPU node by class-aware sharding
    (ref_grid_shares):

    * TST grid, 1536 points: one TST-shaped data set (p = 12, K = 9, nsup = 3, h = 25, gen_lag 4) for
      every point; the share's shape classes (embed_lag x graph-conv layers) are packs whose replicas
      mix the four pretrain / acclimation schedules.  Share `share` is also timed against a control:
      the same packs with every replica on replica 0's schedule (the uniform-pack figure).
    * synthetic grid, 990 data sets: one model config (h = 25, gen_lag 4, DGCNN 16 / 3 / 100, K =
      nsup = numF) per data set; each (K, p) class of the share is a pack with PerReplica data and
      true graphs (sVAR-shaped windows, one seeded set per replica).  See SYN_GRID_NOTE for which grid.

    Rank r of an N-GPU run fits share r (mod 8); the timed regions are max-over-ranks, so with 8 ranks the
    per-grid seconds ARE the node's.  A one-GPU run fits share 0 and then, one after the other on the same
    GPU, the grid's COSTLIEST share (the largest summed cost), and derives the node's figure from the
    slowest share timed: node_fits_per_hour = grid fits x 3600 / max(share seconds) -- a 1-GPU per-share
    timing, no collective (the shares share nothing).

    Every fit runs a fixed schedule scaled 1/10 from the reference's (max_iter 300 -> 30 epochs,
    pretrain / acclimation epochs / 10, rounded up) over 8 training and 2 validation batches of 128
    windows, early stopping disabled so every fit does the same work, per-epoch GC tracking and
    validation on the GPU."""
    import redcliff_amd
    from redcliff_amd import PerReplica, ReplicaPack, fit_packs
    share = rank % 8 if getattr(args, "ref_grid_share", -1) < 0 else args.ref_grid_share
    E, ntr, nva, B = args.ref_grid_epochs, 8, 2, 128
    prof = []
    grids = ref_grid_shares("model" if getattr(args, "ref_grid_model", 0) else "flop")
    out = {"share": "%d of 8 (class-aware shard_grid: %s)" % (share, "min-max runs under REF_GRID_COST" if getattr(
        args, "ref_grid_model", 0) else "FLOP-weighted equal-cost cut, min_piece 32"), "epochs_per_fit": E,
           "train_windows": ntr * B, "val_windows": nva * B}

    def run(packs, warm=True):
        """[(models, opts, train, val, gc)] -> seconds for all packs, fitted concurrently (fit_packs: one
        stream per pack, every pack's epoch enqueued before the host waits; after an untimed 2-epoch
        warm-up fit of a copy of every pack: each shape class's first launches -- kernel loads, LDS
        opt-ins, workspace and data caches -- stay out of the timed region)."""
        if warm:
            import copy
            for m0, o0, tr0, va0, gc0 in packs:
                wm = [copy.deepcopy(m) for m in m0]
                wo = [(torch.optim.Adam(m.gen_model[0].parameters(), lr=1e-4, eps=1e-4, weight_decay=1e-4),
                       torch.optim.Adam(m.gen_model[1].parameters(), lr=1e-4, eps=1e-4, weight_decay=1e-4))
                      for m in wm]
                ReplicaPack(wm, wo).fit(None, tr0, va0, max_iter=2, lookback=10 ** 6, check_every=10 ** 6, GC=gc0)
                del wm, wo
            torch.cuda.synchronize()
        built = [(ReplicaPack(ms, os_), tr, va, gc) for ms, os_, tr, va, gc in packs]

        def go():
            fit_packs([(pk, (None, tr, va), dict(max_iter=E, lookback=10 ** 6, check_every=10 ** 6, GC=gc))
                       for pk, tr, va, gc in built])
        el = timed(go, dist, dev)
        if os.environ.get("REDCLIFF_PACK_PROFILE", "0") != "0":  # host ms per epoch of each pack (replicas.py)
            prof.append([{"R": pk.R, "host_ms_per_epoch": [round(1e3 * float(v), 3) for v in
                                                          np.mean(np.asarray(pk.last_profile), axis=0)]}
                         for pk, _, _, _ in built if pk.last_profile])
        del built
        return el

    # ---- TST grid
    pts, _, _, tshares, tcost = grids["tst"]
    base = CONFIGS["c4"]
    sched = lambda q: (-(-q["pre"] // 10), -(-q["acc"] // 10))  # noqa: E731  (1/10 of the reference's epochs)

    def tst_classes(s):
        classes = {}
        for i in tshares[s]:
            classes.setdefault((pts[i]["lag"], pts[i]["layers"]), []).append(i)
        return classes

    def tst_packs(classes, uniform):
        packs = []
        for (lag, layers), idx in classes.items():
            c = dict(base, F=lag, n=layers, T=lag + 4)
            X, Y = synth(c, (ntr + nva) * B, seed=400 + rank)
            train = [(X[i:i + B], Y[i:i + B]) for i in range(0, ntr * B, B)]
            val = [(X[i:i + B], Y[i:i + B]) for i in range(ntr * B, (ntr + nva) * B, B)]
            rng = np.random.RandomState(8)
            gc = [(rng.rand(c["p"], c["p"], c["L"]) < 0.2).astype(np.float64) for _ in range(c["nsup"])]
            ms, os_ = [], []
            for j, i in enumerate(idx):
                q = pts[i]
                pre, acc = sched(pts[idx[0]] if uniform else q)
                m = build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=7000 + i, pre=pre, acc=acc,
                                forecast=q["forecast"], adj=q["adj"]).to(dev)
                ms.append(m)
                os_.append(adam_pair(m, dict(c, lrA=q["embed_lr"], lrB=q["gen_lr"])))
            packs.append((ms, os_, train, val, gc))
        return packs

    def tst_share(s, control):
        classes = tst_classes(s)
        el = run(tst_packs(classes, False))
        n = len(tshares[s])
        r = {"share": s, "fits": n, "model_seconds": round(tcost[s], 3),
             "packs": [{"embed_lag": k[0], "graph_conv_layers": k[1], "replicas": len(v),
                        "schedules": sorted(set(sched(pts[i]) for i in v))} for k, v in classes.items()],
             "seconds": round(el, 3), "fits_per_hour": round(n * 3600.0 / el, 1)}
        if control:
            el_uni = run(tst_packs(classes, True), warm=False)  # the same shapes: warm
            r.update(uniform_schedule_seconds=round(el_uni, 3),
                     uniform_schedule_fits_per_hour=round(n * 3600.0 / el_uni, 1),
                     mixed_over_uniform_time=round(el / el_uni, 3))
        return r

    # ---- synthetic grid
    kp, _, _, sshares, scost = grids["synthetic"]

    def syn_share(s):
        by = {}
        for i in sshares[s]:
            by.setdefault(kp[i], []).append(i)
        packs = []
        for (K, p), idx in by.items():
            c = _syn_cfg(K, p)
            trains, vals, gcs, ms, os_ = [], [], [], [], []
            for i in idx:
                X, Y = synth(c, (ntr + nva) * B, seed=9000 + i)
                trains.append([(X[j:j + B], Y[j:j + B]) for j in range(0, ntr * B, B)])
                vals.append([(X[j:j + B], Y[j:j + B]) for j in range(ntr * B, (ntr + nva) * B, B)])
                rng = np.random.RandomState(i)
                gcs.append([(rng.rand(p, p, 2) < 0.3).astype(np.float64) for _ in range(K)])
                m = build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=11000 + i, pre=10,
                                acc=10).to(dev)
                ms.append(m)
                os_.append(adam_pair(m, c))
            packs.append((ms, os_, PerReplica(trains), PerReplica(vals), PerReplica(gcs)))
        el = run(packs)
        n = len(sshares[s])
        return {"share": s, "fits": n, "model_seconds": round(scost[s], 3),
                "packs": [{"K": k[0], "p": k[1], "replicas": len(v)} for k, v in by.items()],
                "seconds": round(el, 3), "fits_per_hour": round(n * 3600.0 / el, 1)}

    for name, timer, gcost, n_all in (("tst", lambda s, first: tst_share(s, first), tcost, len(pts)),
                                      ("synthetic", lambda s, first: syn_share(s), scost, len(kp))):
        costliest = int(np.argmax(gcost))
        todo = [share] + ([costliest] if world == 1 and costliest != share else [])
        if world == 1 and getattr(args, "ref_grid_all_shares", False):
            todo = [share] + [s for s in range(8) if s != share]
        runs = []
        for j, s_ in enumerate(todo):
            runs.append(timer(s_, j == 0))
            # progress on stderr (a long all-shares run must not look hung to the GPU harness)
            print("reference_grids: %s share %d: %d fits, %.3f s" % (name, s_, runs[-1]["fits"], runs[-1]["seconds"]),
                  file=sys.stderr, flush=True)
        g = dict(runs[0])
        g["shares_timed"] = runs
        g["costliest_share"] = costliest  # the slowest by the REF_GRID_COST model
        g["share_model_seconds"] = [round(x, 3) for x in gcost]
        slowest = max(r_["seconds"] for r_ in runs)
        g["node_fits_per_hour"] = round(n_all * 3600.0 / slowest, 1)
        g["node_fits_per_hour_basis"] = (
            "%d-GPU run: every rank fits its own share, seconds are max over ranks" % world if world > 1 else
            "1-GPU per-share timing, no collective: %d grid fits x 3600 / the slowest of the timed shares %s "
            "(%.3f s)" % (n_all, [r_["share"] for r_ in runs], slowest))
        out[name] = g
    out["synthetic"]["grid"] = SYN_GRID_NOTE
    if prof:
        out["host_profile"] = {"segments": "enqueue evaluation, enqueue next training epoch, wait for the device, "
                                           "digest the epoch", "runs": prof}
    out["note"] = ("fixed 1/10-scaled schedules (%d epochs; TST pretrain {10, 5} / acclimation {2, 10}; synthetic "
                   "10 / 10), early stopping disabled, 8 x 128 training + 2 x 128 validation windows per fit; the "
                   "packs of a share (one per shape class) run concurrently, one stream each (fit_packs)" % E)
    return out


# --------------------------------------------------------------------------- modes
def mode_fit(args, dev, rank, world, dist, holder):
    from redcliff_amd import _native as nat  # noqa: F401
    c = CONFIGS[args.config]
    B = c["B"]
    eng, plan = single_fit(c, args, dev, rank)
    plan(args.warmup, 0).run()
    extra = preheat(plan, args.warmup, args.preheat_s)
    p_timed = plan(args.steps, args.warmup + extra)
    elapsed = timed(p_timed.run, dist, dev)
    value = world * args.steps * B / elapsed

    out = {"metric": METRIC, "value": round(value, 1), "unit": "windows/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic (D4IC/sVAR-shaped windows; datasets not in image)",
           "preheat": {"seconds": args.preheat_s, "extra_untimed_steps": extra,
                       "note": "untimed steps after the W warm-up steps until the device has been busy this long "
                               "(clock ramp after the host-side setup); the timed region is exactly `steps` steps"},
           "config": {"workload": c["workload"], "global_batch": B * world, "windows_per_step_per_gpu": B,
                      "parallelism": "replicas%d (one independent fit per GPU, no collective)" % world,
                      "ranks": world, "flops_per_window": flops_per_window(c)["total"]}}

    ktimes = None if args.no_kernel_times else kernel_times_of(plan(min(args.steps, 100), 7).run)

    grid = None
    if args.replicas > 1:
        gel, R, gsteps = run_grid(c, args, dev, rank, dist)
        gv = world * R * args.grid_steps * B / gel
        grid = {"replicas_per_gpu": R, "steps": args.grid_steps, "windows_per_s": round(gv, 1),
                "ms_per_step": round(1e3 * gel / args.grid_steps, 4), "speedup_vs_single_fit": round(gv / value, 2),
                "note": "R independent fits (grid points) per GPU, each B=%d windows per step; one launch per kernel "
                        "for all R" % B}
        if not args.no_kernel_times:
            # per-kernel durations with the factor chain on the caller's stream (REDCLIFF_FORK=0, the same
            # bits): on two streams the HIP-event buckets of concurrent kernels overlap and each one
            # over-states its kernel.  The GEMM-shaped embedder's slots are chains of launches
            # (6 products + element-wise kernels), reported but not priced as one kernel.
            fork_env = os.environ.get("REDCLIFF_FORK")
            os.environ["REDCLIFF_FORK"] = "0"
            try:
                gkt = kernel_times_of(gsteps(min(args.grid_steps, 20), 3))
            finally:
                if fork_env is None:
                    del os.environ["REDCLIFF_FORK"]
                else:
                    os.environ["REDCLIFF_FORK"] = fork_env
            grid["roofline"] = roofline_of(gkt, flops_per_window(c), R * B, "%s_r%d" % (args.config, R),
                                           short_factor_kernels(c), chains=("emb_fwd", "emb_bwd"))
            grid["roofline"]["timing"] = ("HIP events per kernel with the factor chain on one stream (REDCLIFF_FORK=0); "
                                          "emb_fwd / emb_bwd are chains of GEMM-embedder launches")
    fph = None
    if args.fit_replicas > 0:
        fph = fits_per_hour(c, args, dev, rank, dist, world)
    refg = None
    if args.ref_grid_epochs > 0 and world <= 8:
        refg = reference_grids(args, dev, rank, world, dist)

    ns = None
    if world == 1 and not args.no_north_star and args.config != "c1k4":
        cn = CONFIGS["c1k4"]
        _, nplan = single_fit(cn, args, dev, rank)
        nplan(args.warmup, 0).run()
        nextra = preheat(nplan, args.warmup, args.preheat_s)
        nsteps = max(args.steps, 50)
        nel = timed(nplan(nsteps, args.warmup + nextra).run, None, dev)
        ns = {"workload": cn["workload"], "windows_per_s": round(nsteps * cn["B"] / nel, 1),
              "ms_per_step": round(1e3 * nel / nsteps, 4), "steps": nsteps, "target_gpu_over_cpu": 50.0}

    c5 = None
    if world == 1 and args.c5_steps > 0:
        c5 = stress_leg(args, dev, rank)

    dpl = None
    dpg = None
    if args.dp_leg_batch > 0 and dist is None and world == 1:
        # one rank: the RCCL group exists only from here on -- a process with an RCCL communicator
        # runs a step's second stream (the split-lead step, forked packs) serialised behind the
        # first (C1(K=4): 0.097 -> 0.132 ms per step, profiles/r04_ns_probe.log), so the legs
        # above ran without one, as a one-GPU user's fits do
        dist = init_group(dev, 1, 0)
        holder["dist"] = dist
    elif args.dp_leg_batch > 0 and dist is not None and world > 1:
        # several ranks: the legs above were coordinated over gloo; the RCCL group of the
        # all-reduce is created now, for this leg only (the same reason)
        dpg = dist.new_group(backend="nccl", device_id=dev)
    if args.dp_leg_batch > 0 and dist is not None:
        # configs[3] beside the replica numbers: ONE TST-shaped fit data-parallel over all ranks
        # (global batch --dp-leg-batch, RCCL all-reduce of the flat gradient per update), so the
        # driver's 1 -> 8 GPU runs record both scaling regimes
        dsteps = max(20, min(args.steps, 200))
        del_, dpo = dp_throughput(args.dp_leg_batch, dsteps, 5, dev, dist, group=dpg)
        dpl = {"global_batch": args.dp_leg_batch, "windows_per_shard": args.dp_leg_batch // world, "ranks": world,
               "updates": dsteps, "windows_per_s": round(dsteps * args.dp_leg_batch / del_, 1),
               "ms_per_update": round(1e3 * del_ / dsteps, 4), "scaling": "strong",
               "allreduce_floats_per_update": int(dpo.PA + dpo.PB),
               "resident_windows_per_rank": getattr(dpo, "resident_windows", None),
               "workload": CONFIGS["c4"]["workload"].replace("B=128", "global B=%d" % args.dp_leg_batch)}

    if rank != 0:
        return None
    if ktimes:
        out["roofline"] = roofline_of(ktimes, flops_per_window(c), B, args.config)
    out["roofline_hbm"] = hbm_roofline(c, eng, 1e3 * elapsed / args.steps, out.get("roofline"))
    out["grid_search"] = grid
    out["fits_per_hour"] = fph
    out["reference_grids"] = refg
    out["data_parallel"] = dpl
    if not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(c, args.cpu_seconds)
        out["gpu_over_cpu"] = round(value / world / out["cpu_baseline"]["value"], 1)
        if fph is not None:
            fph["cpu_baseline"] = cpu_fits_per_hour(c, args.cpu_seconds / 2.0,
                                                    fph["epochs_per_fit"] * (fph["train_windows"] // B))
            fph["gpu_over_cpu"] = round(fph["value"] / world / fph["cpu_baseline"]["value"], 1)
        if ns is not None:
            ns["cpu_baseline"] = cpu_baseline(CONFIGS["c1k4"], args.cpu_seconds * 2.0 / 3.0)
            ns["gpu_over_cpu"] = round(ns["windows_per_s"] / ns["cpu_baseline"]["value"], 1)
    out["north_star_config"] = ns
    out["stress_config"] = c5
    return out


def stress_leg(args, dev, rank):
    """BASELINE configs[4] (p = 64, L = 20, K = 8, h = 25, DGCNN F = 64 / 3 / 100, B = 128): the
    single fit's combined-phase steps (the factor networks on the matrix cores, the GEMM-shaped
    embedder, the two chains on two streams), timed like the headline leg, with the roofline of its
    dominant kernel from HIP events taken with the factor chain on the caller's stream
    (REDCLIFF_FORK=0, the same bits; on two streams concurrent kernels' event buckets overlap) and
    the embedder chains' throughput beside it (chains of launches, not one kernel)."""
    c = CONFIGS["c5"]
    B = c["B"]
    _, plan = single_fit(c, args, dev, rank, nbatch=8)
    plan(5, 0).run()
    extra = preheat(plan, 5, args.preheat_s)
    el = timed(plan(args.c5_steps, 5 + extra).run, None, dev)
    fork_env = os.environ.get("REDCLIFF_FORK")
    os.environ["REDCLIFF_FORK"] = "0"
    try:
        kt = kernel_times_of(plan(min(args.c5_steps, 20), 3).run)
    finally:
        if fork_env is None:
            del os.environ["REDCLIFF_FORK"]
        else:
            os.environ["REDCLIFF_FORK"] = fork_env
    fl = flops_per_window(c)
    roof = roofline_of(kt, fl, B, "c5", False, chains=("emb_fwd", "emb_bwd"))
    roof["timing"] = "HIP events per kernel with the factor chain on one stream (REDCLIFF_FORK=0)"
    chains = {}
    for k in ("emb_fwd", "emb_bwd"):
        if kt.get(k, (0, 0))[0] > 0:
            tf = fl[k] * B / (kt[k][0] * 1e-3) / 1e12
            chains[k] = {"avg_us": round(kt[k][0] * 1e3, 2), "algorithmic_flops": fl[k] * B, "tflops": round(tf, 3),
                         "frac": round(tf / FP32_PEAK_TFLOPS, 6)}
    return {"workload": c["workload"], "windows_per_s": round(args.c5_steps * B / el, 1),
            "ms_per_step": round(1e3 * el / args.c5_steps, 4), "steps": args.c5_steps,
            "flops_per_window": fl["total"], "step_tflops": round(fl["total"] * B * args.c5_steps / el / 1e12, 3),
            "roofline": roof, "embedder_chains": chains}


def dp_throughput(B, steps, warmup, dev, dist, group=None):
    """BASELINE configs[3]: one TST-shaped fit sharded over the ranks (DataParallelFit), global
    batch B per update: (elapsed seconds for `steps` combined-phase updates, the DataParallelFit).
    group: the RCCL group of the all-reduce (default: the world group); timing uses `dist`."""
    import redcliff_amd
    from redcliff_amd.data_parallel import DataParallelFit
    c = dict(CONFIGS["c4"], B=B)
    model = build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=0).to(dev)
    oA, oB = adam_pair(model, c)
    nbatch = 16
    X, Y = synth(c, nbatch * B, seed=100)  # every rank generates the same host data set
    dp = DataParallelFit(model, oA, oB, group=group)
    ds = dp.cache_dataset([(X[i:i + B], Y[i:i + B]) for i in range(0, X.shape[0], B)])  # the rank's shards only
    dp.resident_windows = int(ds["X"].shape[0])

    def run(n, start):
        return lambda: dp.run_steps("combined", ds, [(start + i) % nbatch for i in range(n)])

    run(warmup, 0)()
    return timed(run(steps, warmup), dist, dev), dp


def mode_dp(args, dev, rank, world, dist, holder=None):
    """BASELINE configs[3]: one TST-shaped fit sharded over the ranks (DataParallelFit)."""
    c = dict(CONFIGS["c4"], B=args.dp_batch)
    B = c["B"]
    elapsed, dp = dp_throughput(B, args.steps, args.warmup, dev, dist)
    if rank != 0:
        return None
    value = args.steps * B / elapsed
    return {"metric": METRIC, "value": round(value, 1), "unit": "windows/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (TST/LFP-shaped windows; recordings not in image)",
            "config": {"workload": c["workload"].replace("B=128", "global B=%d" % B), "global_batch": B,
                       "windows_per_step_per_gpu": B / world, "ranks": world,
                       "parallelism": "dp%d (RCCL all-reduce of %d gradient floats per update)"
                                      % (world, dp.PA + dp.PB)}}


def mode_plumbing(args, rank, world, dist):
    """No GPU visible (the build container): check the rank plumbing only -- launch, backend,
    world size, barrier-bracketed timing with the max over ranks.  No throughput is claimed."""
    if dist:
        dist.barrier()
        t = torch.tensor([1.0])
        dist.all_reduce(t)
        assert int(t.item()) == world
    if rank != 0:
        return None
    return {"metric": METRIC, "value": None, "unit": "windows/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True,
            "scaling": "strong" if args.mode == "dp" else "weak", "vs_baseline": None, "dtype": "f32",
            "data": "none: no GPU visible, rank plumbing check only (backend %s)" % ("gloo" if dist else "none"),
            "config": {"workload": CONFIGS["c4" if args.mode == "dp" else args.config]["workload"], "ranks": world,
                       "parallelism": ("dp%d" if args.mode == "dp" else "replicas%d") % world}}


def rank_devices(dist, rank, local, world, dev):
    """[{rank, local_rank, device, name, pci}] of every rank (all-gathered), so the record shows
    which GPU each rank ran on."""
    if dev is None:  # the CPU plumbing check: no device, the process identifies the rank
        me = {"rank": rank, "local_rank": local, "device": "cpu", "pid": os.getpid()}
    else:
        props = torch.cuda.get_device_properties(dev)
        me = {"rank": rank, "local_rank": local, "device": dev.index, "name": props.name,
              "pci": "%s:%s:%s" % (getattr(props, "pci_domain_id", "?"), getattr(props, "pci_bus_id", "?"),
                                   getattr(props, "pci_device_id", "?"))}
    if dist is None or world == 1:
        return [me]
    allr = [None] * world
    dist.all_gather_object(allr, me)
    return allr


# --------------------------------------------------------------------------- launch
def init_group(dev, world, local, coordination=False):
    """torch.distributed over RCCL ("nccl") on the GPU, bound to this rank's device (no guessing the
    device from the global rank), or gloo for the CPU plumbing check; 127.0.0.1 rendezvous.
    coordination=True: a gloo group for the barriers and the max-over-ranks timing of --mode fit
    (its legs run no collective on the data path; the data-parallel leg makes its own RCCL group)."""
    import torch.distributed as dist
    kw = {}
    if dev is not None:
        torch.cuda.set_device(dev)
        if not coordination:
            kw["device_id"] = dev
    backend = "gloo" if (dev is None or coordination) else "nccl"
    if world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        dist.init_process_group(backend, rank=0, world_size=1, **kw)
    else:
        dist.init_process_group(backend, **kw)
    return dist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """Start n ranks of this script through torch.distributed.run (127.0.0.1), before any GPU
    call in this process, and return their exit status."""
    argv = [a for a in sys.argv[1:]]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--mode", default="fit", choices=("fit", "dp"))
    ap.add_argument("--config", default="d4ic", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--preheat-s", type=float, default=0.3,
                    help="untimed device-busy seconds after the warm-up steps (0: none)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-times", action="store_true")
    ap.add_argument("--no-north-star", action="store_true")
    # 128 grid points per GPU: the reference's grids (1,536 combinations, or the 990-task synthetic list,
    # SURVEY.md 8(d)) give every one of 8 GPUs well over 128 fits; measured on the current build:
    # R = 32 / 64 / 128 -> 8.4 / 9.2 / 9.9 M windows/s and 0.24 / 0.53 / 0.73 M fits/hour
    ap.add_argument("--replicas", type=int, default=128, help="grid-search replicas packed per GPU (1: skip)")
    ap.add_argument("--grid-steps", type=int, default=100)
    ap.add_argument("--fit-replicas", type=int, default=128, help="packed whole fits for fits/hour (0: skip)")
    ap.add_argument("--fit-epochs", type=int, default=40)
    ap.add_argument("--fit-train-batches", type=int, default=8)
    ap.add_argument("--ref-grid-epochs", type=int, default=30,
                    help="epochs per fit of the reference-grid fits/hour leg (0: skip)")
    ap.add_argument("--ref-grid-share", type=int, default=-1,
                    help="which 8-GPU share the reference-grid leg fits (default: the rank's)")
    ap.add_argument("--ref-grid-model", type=int, default=0,
                    help="1: shares cut by the REF_GRID_COST min-max rule (A/B); 0: the FLOP-weighted equal-cost cut")
    ap.add_argument("--ref-grid-all-shares", action="store_true",
                    help="one GPU: time all 8 shares of each reference grid (default: the share and the costliest)")
    ap.add_argument("--c5-steps", type=int, default=20,
                    help="combined-phase steps of the configs[4] stress leg at N = 1 (0: skip)")
    ap.add_argument("--dp-batch", type=int, default=128, help="global batch of --mode dp")
    # 512 = the most windows one launch takes (Bmax), so one rank can run the same global batch
    ap.add_argument("--dp-leg-batch", type=int, default=512,
                    help="global batch of the data-parallel leg of --mode fit (0: skip)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        import __graft_entry__
        __graft_entry__.build()  # once, in the parent (compiling touches no GPU); the ranks find it current
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cuda = torch.cuda.is_available()
    dist = None
    # one rank in --mode fit: the group for the data-parallel leg is created when that leg runs (mode_fit)
    if world > 1 or args.mode == "dp" or (args.dp_leg_batch > 0 and not cuda):
        dist = init_group(torch.device("cuda", local % max(torch.cuda.device_count(), 1)) if cuda else None, world,
                          local, coordination=(args.mode == "fit"))
        seen = dist.get_world_size()
        if seen != world or (args.gpus > 1 and seen != args.gpus):
            raise SystemExit("world size %d != --gpus %d / WORLD_SIZE %d" % (seen, args.gpus, world))
        world = seen
    if not cuda:
        devices = rank_devices(dist, rank, local, world, None)
        out = mode_plumbing(args, rank, world, dist)
        if out is not None:
            out["config"]["rank_devices"] = devices
            out["config"]["world_size"] = world
            print(json.dumps(out), flush=True)
        if dist:
            dist.destroy_process_group()
        return
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))  # (more ranks than GPUs: rehearsal)
    torch.cuda.set_device(dev)

    # the library is built in-tree (a no-op when current); under an external launcher only the
    # first local rank builds while the others wait, so no two ranks write the .so at once
    if local == 0:
        import __graft_entry__
        __graft_entry__.build()
    if dist is not None:
        dist.barrier()
    devices = rank_devices(dist, rank, local, world, dev)
    holder = {"dist": dist}
    out = (mode_dp if args.mode == "dp" else mode_fit)(args, dev, rank, world, dist, holder)
    if out is not None:
        out["config"]["rank_devices"] = devices
        out["config"]["world_size"] = world
        print(json.dumps(out), flush=True)
    if holder["dist"]:
        holder["dist"].destroy_process_group()


if __name__ == "__main__":
    main()
