"""The packed fit's per-epoch evaluation launches in isolation (R replicas, D4IC shapes): the GC
norms, the embedder for GC tracking, the GC-progress metrics and statistics, validation values.
Prints the per-call device time of each (HIP events); run under rocprofv3 for per-kernel stats
or PMC counters (kernel names k_gc_norms, k_gc_dots, k_gc_progress, k_cos_values, ...).

    python scripts/eval_kernels.py [--replicas 128] [--reps 20]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="d4ic")
    ap.add_argument("--replicas", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    import bench
    import redcliff_amd
    from redcliff_amd import metrics as M
    from redcliff_amd.fit_loop import conditional_gc_estimates
    c = bench.CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    R, B = args.replicas, c["B"]
    models, opts = [], []
    for i in range(R):
        m = bench.build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=900 + i).to(dev)
        models.append(m)
        opts.append(bench.adam_pair(m, c))
    pack = redcliff_amd.ReplicaPack(models, opts)
    X, Y = bench.synth(c, 2 * B, seed=5)
    val = pack.cache_dataset([(X[:B], Y[:B]), (X[B:], Y[B:])])
    pack._workspace(B, val["T"])
    rng = np.random.RandomState(7)
    true_gc = [(rng.rand(c["p"], c["p"], c["L"]) < 0.2).astype(np.float64) for _ in range(c["K"])]
    m0 = models[0]
    Xv = val["X"][:min(B, m0.MAX_NUM_SAMPS_FOR_GC_PROGRESS_TRACKING), :m0.Lmax, :]
    ls = min(m0.gen_lag, m0.embed_lag)
    p, nsup = c["p"], c["nsup"]

    def ev_time(fn, reps):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return round(1e3 * a.elapsed_time(b) / reps, 2)

    def estimates():
        w_raw = pack.embed_raw(Xv)
        w = torch.sigmoid(m0.factor_score_embedder.sigmoid_eccentricity_coeff * w_raw) \
            if m0.factor_score_embedder.use_sigmoid_restriction else w_raw
        G, G0 = pack.gc_norms()
        A = pack.emb[:, :p * p].view(R, p, p)
        return conditional_gc_estimates(w, G, G0, A, nsup, ls, m0.primary_gc_est_mode)

    est_t, nolag_t = estimates()
    Ra, S = est_t.shape[0], est_t.shape[1]
    out = {"config": args.config, "replicas": R, "us_per_call": {
        "gc_norms": ev_time(pack.gc_norms, args.reps),
        "embed_raw": ev_time(lambda: pack.embed_raw(Xv), args.reps),
        "estimates (embed + norms + torch)": ev_time(estimates, args.reps),
        "gc_progress_values": ev_time(lambda: M.gc_progress_values(true_gc, est_t.reshape(Ra * S, *est_t.shape[2:]),
                                                                   0.1, 1., 1., host=False), args.reps),
        "gc_track_values": ev_time(lambda: M.gc_track_values(est_t, nolag_t, host=False), args.reps),
        "validation values (2 batches)": ev_time(lambda: pack._values(val, host=False), args.reps)}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
