"""Where the wall clock of a packed grid-search fit (ReplicaPack.fit, the fits/hour unit of work)
goes: training launches vs per-epoch GC tracking (device metrics + host trackers) vs validation
vs best-model snapshots.  Same workload as bench.py's fits_per_hour leg; prints one JSON line.
--gc-kernel also times redcliff_gc_progress alone (HIP events) at the config's shapes."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))

import bench  # noqa: E402


def gc_kernel_time(c, reps=20):
    from redcliff_amd import metrics as M
    p, K, L = c["p"], c["K"], c["L"]
    S = c["nsup"]
    rng = np.random.RandomState(0)
    GC = [(rng.rand(p, p, L) < 0.2).astype(np.float64) for _ in range(K)]
    est = torch.from_numpy(rng.rand(S, K, p, p, L).astype(np.float32)).cuda()
    M.gc_progress_values(GC, est)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    for _ in range(reps):
        M.gc_progress_values(GC, est)
    b.record()
    torch.cuda.synchronize()
    return {"S": S, "G": K, "p": p, "Lt": L, "ms_per_call_events": a.elapsed_time(b) / reps,
            "ms_per_call_wall": 1e3 * (time.perf_counter() - t0) / reps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="d4ic")
    ap.add_argument("--replicas", type=int, default=32)
    ap.add_argument("--epochs", type=int, default=12)
    ap.add_argument("--train-batches", type=int, default=8)
    ap.add_argument("--gc-kernel", action="store_true")
    ap.add_argument("--cprofile", action="store_true", help="host-side cProfile of one unwrapped packed fit")
    ap.add_argument("--host-split", action="store_true",
                    help="one more fit with REDCLIFF_PACK_PROFILE=1: host ms per epoch enqueueing the evaluation, "
                         "enqueueing the next training epoch, waiting for the device, digesting the epoch")
    ap.add_argument("--torch-eval", action="store_true",
                    help="comparison: the end-of-fit module modes set with torch's recursive .eval()")
    args = ap.parse_args()
    import redcliff_amd
    from redcliff_amd import fit_loop, replicas
    from redcliff_amd import metrics as M
    if args.torch_eval:
        def torch_eval_modes(models, dicts=None):
            for m in models:
                m.factor_score_embedder.eval()
                for f in m.factors:
                    f.eval()
        replicas._eval_modes = torch_eval_modes
    c = bench.CONFIGS[args.config]
    B, R, E = c["B"], args.replicas, args.epochs
    ntr, nva = args.train_batches, 2
    X, Y = bench.synth(c, (ntr + nva) * B, seed=300)
    train = [(X[i:i + B], Y[i:i + B]) for i in range(0, ntr * B, B)]
    val = [(X[i:i + B], Y[i:i + B]) for i in range(ntr * B, (ntr + nva) * B, B)]
    rng = np.random.RandomState(7)
    true_gc = [(rng.rand(c["p"], c["p"], c["L"]) < 0.2).astype(np.float64) for _ in range(c["K"])]
    pre, acc = max(1, E // 5), max(1, E // 10)

    def make_pack():
        models, opts = [], []
        for i in range(R):
            m = bench.build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=5000 + i, pre=pre,
                                  acc=acc).cuda()
            models.append(m)
            opts.append(bench.adam_pair(m, c))
        return redcliff_amd.ReplicaPack(models, opts)

    def fit(pack):
        pack.fit(None, train, val, max_iter=E, lookback=10 ** 6, check_every=10 ** 6, GC=true_gc)

    fit(make_pack())  # warm-up (builds, caches)
    pack = make_pack()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fit(pack)
    torch.cuda.synchronize()
    unwrapped = time.perf_counter() - t0
    host_split = None
    if args.host_split:
        os.environ["REDCLIFF_PACK_PROFILE"] = "1"
        pack = make_pack()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fit(pack)
        torch.cuda.synchronize()
        tot = time.perf_counter() - t0
        os.environ.pop("REDCLIFF_PACK_PROFILE")
        pr = np.asarray(pack.last_profile) * 1e3  # [epochs][4] ms
        phases = {"pretrain": (0, pre), "acclimation": (pre, pre + acc), "combined": (pre + acc, E)}
        host_split = {"fit_s": round(tot, 4), "columns": ["enqueue_eval", "enqueue_train", "wait_device", "digest"]}
        host_split["before_loop_ms"], host_split["loop_ms"], host_split["after_loop_ms"] = [
            round(1e3 * x, 2) for x in pack.last_profile_edges]
        for k, (a, b) in phases.items():
            host_split[k] = [round(float(x), 3) for x in pr[a:b].mean(axis=0)] if b > a else None
    if args.cprofile:
        import cProfile
        import pstats
        pack = make_pack()
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        pr.enable()
        fit(pack)
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(40)
        pstats.Stats(pr).sort_stats("cumulative").print_stats(40)

    times = {}

    def wrap(owner, name, key):
        f = getattr(owner, name)

        def g(*a, **k):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = f(*a, **k)
            torch.cuda.synchronize()
            times[key] = times.get(key, 0.0) + time.perf_counter() - t
            return r
        setattr(owner, name, g)
        return f

    saved = []
    for n in ("run_epoch", "embed_raw", "gc_norms", "_values", "cache_dataset"):
        saved.append((replicas.ReplicaPack, n, wrap(replicas.ReplicaPack, n, "pack." + n)))
    for n in ("gc_progress", "step", "validation", "train_confusion"):
        saved.append((fit_loop.FitTracker, n, wrap(fit_loop.FitTracker, n, "tracker." + n)))
    for n in ("gc_progress_values", "track_roc_stats_from_values", "track_deltacon_stats_from_values",
              "track_cosine_stats_batched", "track_l1_stats"):
        saved.append((M, n, wrap(M, n, "M." + n)))
    saved.append((replicas, "conditional_gc_estimates",
                  wrap(replicas, "conditional_gc_estimates", "conditional_gc_estimates")))
    saved.append((replicas._PackBest, "copy_marked", wrap(replicas._PackBest, "copy_marked", "best.copy_marked")))
    pack = make_pack()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fit(pack)
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    for owner, name, f in saved:
        setattr(owner, name, f)
    out = {"config": args.config, "replicas": R, "epochs": E, "train_batches": ntr, "val_batches": nva,
           "unwrapped_fit_s": round(unwrapped, 4), "unwrapped_per_epoch_ms": round(1e3 * unwrapped / E, 2),
           "fits_per_hour_1gpu": round(R * 3600.0 / unwrapped, 1),
           "wrapped_per_epoch_ms": round(1e3 * total / E, 2),
           "breakdown_ms_per_epoch": dict((k, round(1e3 * v / E, 3)) for k, v in sorted(times.items()))}
    if args.gc_kernel:
        out["gc_progress_kernel"] = gc_kernel_time(c)
    if host_split is not None:
        out["host_split_ms_per_epoch"] = host_split
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
