"""Run-to-run determinism of small synthetic-grid shapes on the packed-grid kernel paths
(REDCLIFF_FAC_PATH=mfma, REDCLIFF_EMB_PATH=gemm): the same fit twice (one replica) and the same pack
twice must give the same bits; then the pack against the single fits.  Prints one line per check.

    python scripts/determinism_probe.py [--shapes 2x3,1x12,1x3,10x6] [--epochs 7]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="2x3,1x12,1x3,10x6")
    ap.add_argument("--epochs", type=int, default=7)
    ap.add_argument("--hist", action="store_true", help="the pack test's order and history comparison")
    ap.add_argument("--steps-only", action="store_true", help="plain batch_update epochs instead of fit()")
    args = ap.parse_args()
    os.environ.setdefault("REDCLIFF_FAC_PATH", "mfma")
    os.environ.setdefault("REDCLIFF_EMB_PATH", "gemm")
    import redcliff_amd
    from redcliff_amd import PerReplica, ReplicaPack
    from test_gpu_pack_fit import true_graphs

    for shp in args.shapes.split(","):
        K, p = [int(x) for x in shp.split("x")]

        def model(seed):
            coeff = {"FORECAST_COEFF": 10.0, "FACTOR_SCORE_COEFF": 100.0,
                     "FACTOR_COS_SIM_COEFF": 1.0 / (sum(range(1, K)) if K > 1 else 1.0), "FACTOR_WEIGHT_L1_COEFF": 1e-3,
                     "FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF": 0.0, "ADJ_L1_REG_COEFF": 0.1 / K / np.sqrt(p * p - 1.0),
                     "DAGNESS_REG_COEFF": 0.0, "DAGNESS_LAG_COEFF": 0.0, "DAGNESS_NODE_COEFF": 0.0}
            eargs = [("num_features_per_node", 16), ("num_graph_conv_layers", 3), ("num_hidden_nodes", 100),
                     ("sigmoid_eccentricity_coeff", 10.0)]
            torch.manual_seed(seed)
            return redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing(
                p, 4, [25], 16, [0], 4, 1, K, K, coeff, False, "DGCNN", eargs, "conditional_factor_fixed_embedder",
                "apply_factor_weights_after_sim_completion", num_sims=1,
                training_mode="pretrain_embedder_then_acclimate_factors_then_combined", num_pretrain_epochs=2,
                num_acclimation_epochs=1).cuda()

        def dataset(seed, N):
            rng = np.random.RandomState(seed)
            X = rng.randn(N, 24, p).astype(np.float32)
            Y = np.zeros((N, K, 24), np.float32)
            Y[np.arange(N), rng.randint(0, K, N), :] = 1.0
            X, Y = torch.from_numpy(X), torch.from_numpy(Y)
            return [(X[i:i + 64], Y[i:i + 64]) for i in range(0, N, 64)]
        R = 3
        trains = [dataset(70 + r, 64 * 2 + 24) for r in range(R)]
        vals = [dataset(80 + r, 96) for r in range(R)]
        gcs = [true_graphs(K, p, 2, seed=90 + r) for r in range(R)]
        kw = dict(lookback=1, check_every=1, deltaConEps=0.1, verbose=0, stopping_criteria_forecast_coeff=10.,
                  stopping_criteria_factor_coeff=100., stopping_criteria_cosSim_coeff=1.)

        def opts(m):
            return (torch.optim.Adam(m.gen_model[0].parameters(), lr=5e-4, eps=1e-4, weight_decay=1e-4),
                    torch.optim.Adam(m.gen_model[1].parameters(), lr=5e-4, eps=1e-4, weight_decay=1e-4))

        def single(r):
            m = model(100 + r)
            oA, oB = opts(m)
            if args.steps_only:
                for ep in range(args.epochs):
                    for bi, (Xb, Yb) in enumerate(trains[r]):
                        m.batch_update(ep, bi, Xb, Yb, oA, oB, 1)
            else:
                m.fit(None, trains[r], oA, oB, 4, 1, 1, args.epochs, vals[r], GC=gcs[r], **kw)
            torch.cuda.synchronize()
            return {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}

        def packed():
            ms = [model(100 + r) for r in range(R)]
            pk = ReplicaPack(ms, [opts(m) for m in ms])
            if args.steps_only:
                ds = pk.cache_dataset(PerReplica(trains))
                for ep in range(args.epochs):
                    pk.run_epoch(ep, ds)
            else:
                pk.fit(None, PerReplica(trains), PerReplica(vals), args.epochs, GC=PerReplica(gcs), **kw)
            torch.cuda.synchronize()
            return [{k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()} for m in ms]

        if args.hist:  # the test's order: solo fits r = 0, 1, 2, then the pack; histories entry by entry
            HK = ("avg_forecasting_loss", "avg_factor_loss", "avg_factor_cos_sim_penalty", "avg_fw_l1_penalty",
                  "avg_adj_penalty", "avg_combo_loss")
            solo = []
            for r in range(R):
                m = model(100 + r)
                oA, oB = opts(m)
                m.fit(None, trains[r], oA, oB, 4, 1, 1, args.epochs, vals[r], GC=gcs[r], **kw)
                torch.cuda.synchronize()
                solo.append(m)
            ms = [model(100 + r) for r in range(R)]
            pk = ReplicaPack(ms, [opts(m) for m in ms])
            pk.fit(None, PerReplica(trains), PerReplica(vals), args.epochs, GC=PerReplica(gcs), **kw)
            torch.cuda.synchronize()
            for r in range(R):
                ha, hb = solo[r].fit_history, ms[r].fit_history
                print("K=%d p=%d r=%d best_it solo %s pack %s stopped %s %s" % (K, p, r, ha["best_it"], hb["best_it"],
                                                                       ha.get("stopped_at"), hb.get("stopped_at")))
                for k in HK:
                    a, b = list(ha[k]), list(hb[k])
                    bad = [(i, float(x), float(y)) for i, (x, y) in enumerate(zip(a, b)) if not (x == y)]
                    if bad or len(a) != len(b):
                        print("   %s len %d/%d differ at %s" % (k, len(a), len(b), bad[:4]))
                sa = {k: v.detach().cpu().numpy() for k, v in solo[r].state_dict().items()}
                sb = {k: v.detach().cpu().numpy() for k, v in ms[r].state_dict().items()}
                print("   state arrays differing:", [k for k in sa if not np.array_equal(sa[k], sb[k], equal_nan=True)][:6])
            continue

        def ndiff(a, b):
            return [k for k in a if not np.array_equal(a[k], b[k], equal_nan=True)]
        s1, s2 = single(1), single(1)
        p1, p2 = packed(), packed()
        print("K=%d p=%d  single twice: %d differ %s" % (K, p, len(ndiff(s1, s2)), ndiff(s1, s2)[:4]), flush=True)
        print("K=%d p=%d  pack twice:   %s" % (K, p, [len(ndiff(a, b)) for a, b in zip(p1, p2)]), flush=True)
        print("K=%d p=%d  pack vs single (replica 1): %d differ %s" % (K, p, len(ndiff(p1[1], s1)), ndiff(p1[1], s1)[:6]),
              flush=True)


if __name__ == "__main__":
    main()
