#!/usr/bin/env python
"""REDCLIFF-S cMLP factor-model fitting on MI355X: fused fwd+bwd windows/sec.

A "step" is one REDCLIFF-S batch_update in the combined training phase (embedder +
K x p factor networks forward, conditional-GC penalties, backward, Adam on both
optimizer groups) over one batch of B=128 synthetic windows resident in HBM.
Default workload = BASELINE.json configs[1]: REDCLIFF-S w/ state smoothing, D4IC-shaped
(p=10 channels, gen_lag 4, 4 factors, hidden 100, DGCNN F=20 / 2 layers / 30 hidden,
windows of 21 steps, labels (N, K, 1)); D4IC itself is not in the image, so the windows
are synthetic with the same shapes.

    python bench.py [--gpus N --steps K --warmup W]      (N>1: one rank per GPU via torchrun)

Multi-GPU: every rank runs an independent fit (grid-search replicas shard one per GPU,
no collective); value = all windows processed / max-over-ranks time ("scaling": "weak").
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))

FP32_PEAK_TFLOPS = 157.3  # MI355X dense FP32 (vector == f32 MFMA rate), MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    # BASELINE.json configs[1]: D4IC-shaped, 4 factors (train/REDCLIFF_S_CMLP_Smooth_d4IC_BSCgs4ParsimSmo0_cached_args.txt)
    "d4ic": dict(p=10, L=4, K=4, nsup=4, h=100, F=20, n=2, H=30, B=128, T=21, label_T=1, lrA=2e-4, lrB=5e-4,
                 workload="REDCLIFF-S cMLP w/ state smoothing, D4IC-shaped (p=10, gen_lag=4, K=4, h=100, "
                          "DGCNN F=20/2 layers/30 hidden), combined-phase batch_update, B=128"),
    # north-star ratio config: 10 channels / 5 lags / 4 factors (synthetic sVAR shapes)
    "c1k4": dict(p=10, L=5, K=4, nsup=4, h=25, F=16, n=3, H=100, B=128, T=100, label_T=100, lrA=5e-4, lrB=5e-4,
                 workload="REDCLIFF-S cMLP w/ state smoothing, synthetic sVAR (p=10, gen_lag=5, K=4, h=25, "
                          "DGCNN F=16/3 layers/100 hidden), combined-phase batch_update, B=128"),
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



def roofline_of(ktimes, fl, windows_per_launch, with_traffic):
    """Roofline object of the dominant kernel: algorithmic FLOPs per launch (SURVEY 8(d)
    per-window counts x the windows one launch processes) / its average HIP-event duration.
    Timing slots: "emb_fwd" = k_forward (embedder + vector-path factor forward in one launch)
    or the GEMM embedder's forward chain; on the matrix-core path "fac_fwd" = k_xwin +
    k_fac_fwd_mfma, "fac_mix" = k_fac_mix, "fac_bwd" = k_fac_bwd_mfma.  With two kernel chains
    on two streams the slots overlap in time (the step is shorter than their sum)."""
    fl = dict(fl)
    mfma = ktimes.get("fac_mix", (0, 0))[1] > 0
    if mfma:  # k_fac_mix carries the penalty terms, k_fac_bwd_mfma the dW0 contraction
        fl["fac_mix"] = fl["pen"]
        fl["fac_bwd"] -= fl["pen"]
    elif ktimes.get("fac_fwd", (0, 0))[1] == 0:
        fl["emb_fwd"] += fl["fac_fwd"]
    dom = max((k for k in ktimes if k in fl and k != "supports"), key=lambda k: ktimes[k][0])
    avg_ms = ktimes[dom][0]
    flops = fl.get(dom, 0) * windows_per_launch
    achieved = flops / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    kname = {"emb_fwd": "k_forward", "fac_fwd": "k_fac_fwd_mfma", "fac_bwd": "k_fac_bwd_mfma" if mfma else "k_fac_bwd",
             "emb_bwd": "k_emb_bwd", "emb_final": "k_emb_final", "fac_mix": "k_fac_mix"}[dom]
    return {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 4), "peak": FP32_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / FP32_PEAK_TFLOPS, 6),
            "traffic": pmc_traffic(kname) if with_traffic else None,
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


def build_model(cls, c, seed):
    K, p = c["K"], c["p"]
    denom = sum(float(i) for i in range(1, K)) if K > 1 else 1.0
    coeff = {"FORECAST_COEFF": 10.0, "FACTOR_SCORE_COEFF": 100.0, "FACTOR_COS_SIM_COEFF": 1.0 / denom,
             "FACTOR_WEIGHT_L1_COEFF": 1e-3, "FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF": 0.0,
             "ADJ_L1_REG_COEFF": 0.1 / K / np.sqrt(p * p - 1.0), "DAGNESS_REG_COEFF": 0.0,
             "DAGNESS_LAG_COEFF": 0.0, "DAGNESS_NODE_COEFF": 0.0}
    eargs = [("num_features_per_node", c["F"]), ("num_graph_conv_layers", c["n"]), ("num_hidden_nodes", c["H"]),
             ("sigmoid_eccentricity_coeff", 10.0)]
    torch.manual_seed(seed)
    return cls(p, c["L"], [c["h"]], c["F"], [0], c["L"], 1, K, c["nsup"], coeff, False, "DGCNN", eargs,
               "conditional_factor_fixed_embedder", "apply_factor_weights_after_sim_completion", num_sims=1,
               training_mode="pretrain_embedder_then_acclimate_factors_then_combined", num_pretrain_epochs=1,
               num_acclimation_epochs=1)


def adam_pair(m, c):
    oA = torch.optim.Adam(m.gen_model[0].parameters(), lr=c["lrA"], betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    oB = torch.optim.Adam(m.gen_model[1].parameters(), lr=c["lrB"], betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    return oA, oB


def cpu_baseline(c, seconds):
    """The oracle (CPU restatement keeping the reference's op structure) on the host cores."""
    from oracle.redcliff_oracle import OracleREDCLIFF
    threads = int(os.environ.get("REDCLIFF_CPU_THREADS", min(16, os.cpu_count() or 1)))
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
    dt = time.perf_counter() - t0
    return {"value": round(n * c["B"] / dt, 2), "unit": "windows/s", "cores": threads, "kind": "port",
            "sample": "%d combined-phase batch_updates of B=%d (%.1f s) with oracle/redcliff_oracle.py "
                      "(reference op structure: per-sample loops, autograd, torch.optim.Adam) on %d threads"
                      % (n, c["B"], dt, threads)}


PMC_CONFIG = "d4ic"  # the configuration scripts/profile_pmc.sh collects the counters on


def pmc_traffic(kernel_name, launches_hint=None):
    """HBM bytes per launch of ``kernel_name`` from committed rocprofv3 PMC summaries
    (profiles/*pmc*.csv), FETCH_SIZE x 2 (gfx950 under-count, MI355X_MICROARCH.md HBM) + WRITE_SIZE."""
    import csv
    import glob
    fetch, write = None, None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*counter_collection*.csv"))):
        vals = {}
        with open(path) as f:
            for row in csv.DictReader(f):
                if kernel_name not in row.get("Kernel_Name", ""):
                    continue
                vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
        if "FETCH_SIZE" in vals:
            fetch = float(np.mean(vals["FETCH_SIZE"]))
        if "WRITE_SIZE" in vals:
            write = float(np.mean(vals["WRITE_SIZE"]))
    if fetch is None or write is None:
        return None
    return (2.0 * fetch + write) * 1024.0  # counters are in KiB


def run_grid(c, args, dev, rank, dist):
    """Time args.grid_steps combined-phase steps of R packed grid-search replicas."""
    import redcliff_amd
    K, p = c["K"], c["p"]
    R = args.replicas
    models, opts = [], []
    for i in range(R):
        m = build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=1000 * rank + i).to(dev)
        # vary what the reference grid varies (train/...gsSmooth1.py:278-309): lrs and coefficients
        m.FORECAST_COEFF = (10.0, 1.0)[i % 2]
        m.ADJ_L1_REG_COEFF = (0.1, 0.01)[(i // 2) % 2] / K / np.sqrt(p * p - 1.0)
        cc = dict(c, lrA=(5e-4, 1e-4)[(i // 4) % 2], lrB=(5e-4, 1e-4)[(i // 8) % 2])
        models.append(m)
        opts.append(adam_pair(m, cc))
    pack = redcliff_amd.ReplicaPack(models, opts)
    nbatch = 8
    X, Y = synth(c, nbatch * c["B"], seed=200 + rank)
    ds = pack.cache_dataset([(X[i:i + c["B"]], Y[i:i + c["B"]]) for i in range(0, X.shape[0], c["B"])])

    def steps(n, start):
        idx = (np.arange(n) + start) % nbatch
        pack.run_steps(["combined"], ds, ds["rows"][idx], ds["sizes"][idx],
                       ds["stats"][torch.as_tensor(idx, device=dev)].contiguous())

    steps(5, 0)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps(args.grid_steps, 5)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el, R, steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--config", default="d4ic", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-times", action="store_true")
    ap.add_argument("--replicas", type=int, default=32, help="grid-search replicas packed per GPU (1: skip)")
    ap.add_argument("--grid-steps", type=int, default=100)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    if world == 1:
        import __graft_entry__
        __graft_entry__.build()  # no-op when the in-tree library is up to date
    import redcliff_amd
    from redcliff_amd import _native as nat

    c = CONFIGS[args.config]
    B = c["B"]
    # independent fit per rank (grid-search replica): its own seed and its own data
    model = build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=rank).to(dev)
    oA, oB = adam_pair(model, c)
    nbatch = 32
    X, Y = synth(c, nbatch * B, seed=100 + rank)
    loader = [(X[i:i + B], Y[i:i + B]) for i in range(0, X.shape[0], B)]
    eng = model.engine()
    ds = eng.cache_dataset(loader)
    d = eng.workspace(ds["Bmax"], ds["T"])

    def run(nsteps, start):
        idx = (np.arange(nsteps) + start) % nbatch
        stats = ds["stats"][torch.as_tensor(idx, device=dev)].contiguous()
        eng.run_steps(["combined"], ds["X"], ds["lab"], stats, d, ds["rows"][idx], ds["sizes"][idx], oA, oB)

    run(args.warmup, 0)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps, args.warmup)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    windows = world * args.steps * B
    value = windows / elapsed

    # grid-search replicas packed into one launch: R fits of the same shape
    # with different seeds / coefficients / learning rates, stepped together on this GPU
    grid = None
    if args.replicas > 1:
        grid_elapsed, R, grid_steps_fn = run_grid(c, args, dev, rank, dist)
        gsteps = args.grid_steps
        grid = {"replicas_per_gpu": R, "steps": gsteps,
                "windows_per_s": round(world * R * gsteps * B / grid_elapsed, 1),
                "ms_per_step": round(1e3 * grid_elapsed / gsteps, 4),
                "speedup_vs_single_fit": round((world * R * gsteps * B / grid_elapsed) / value, 2),
                "note": "R independent fits (grid points) per GPU, each B=%d windows per step; one launch per kernel "
                        "for all R" % B}

    # per-kernel device time over the same kind of steps (HIP events on the launch stream)
    ktimes = None
    if not args.no_kernel_times:
        nat.kernel_timing(True)
        nk = min(args.steps, 100)
        run(nk, 7)
        torch.cuda.synchronize()
        kt = nat.kernel_times()
        nat.kernel_timing(False)
        ktimes = dict((k, (ms / n if n else 0.0, n)) for k, (ms, n) in kt.items())

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    fl = flops_per_window(c)
    roof = roofline_of(ktimes, fl, B, args.config == PMC_CONFIG) if ktimes else None
    if grid is not None and not args.no_kernel_times:
        # the same kernel-level roofline for the packed launch: one launch carries R * B windows
        nat.kernel_timing(True)
        grid_steps_fn(min(args.grid_steps, 20), 3)
        torch.cuda.synchronize()
        gkt = nat.kernel_times()
        nat.kernel_timing(False)
        gkt = dict((k, (ms / n if n else 0.0, n)) for k, (ms, n) in gkt.items())
        grid["roofline"] = roofline_of(gkt, flops_per_window(c), grid["replicas_per_gpu"] * B, False)
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(c, args.cpu_seconds)
    out = {
        "metric": "cMLP-factor fwd+bwd windows/sec/GPU; grid-search fits/hour on 8 GPUs",
        "value": round(value, 1), "unit": "windows/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic (D4IC/sVAR-shaped windows; datasets not in image)",
        "config": {"workload": c["workload"], "global_batch": B * world, "windows_per_step_per_gpu": B,
                   "parallelism": "replicas%d (one independent fit per GPU, no collective)" % world,
                   "flops_per_window": fl["total"]},
        "roofline": roof, "cpu_baseline": cpu, "grid_search": grid,
    }
    if cpu:
        out["gpu_over_cpu"] = round(value / world / cpu["value"], 1)
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
