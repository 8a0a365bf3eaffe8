"""Generate tests/golden/eval_pipeline.npz from the REFERENCE's evaluation functions
(run in the build container only; /root/reference is not on the GPU box).

    python tests/golden/make_eval_golden.py

Inputs are seeded synthetic GC estimates / true graphs (p = 10 with lag axes, quantised
scores so ties occur, plus the reference's edge cases).  Outputs are what the reference
returns for them:
  * general_utils/metrics.py  compute_optimal_f1, compute_f1, sensitivity / specificity /
    LR+ / LR-, deltacon0(make_graphs_undirected=True/False);
  * evaluate/eval_utils.py    compute_OptimalF1_stats_betw_two_gc_graphs,
    compute_f1_stats_betw_two_gc_graphs, compute_key_stats_betw_two_gc_graphs,
    get_combined_gc_representations_across_factors;
  * general_utils/misc.py     sort_unsupervised_estimates (return_sorting_inds=True);
  * the factor-level statistics of perform_system_level_estimation_evaluation_of_cv_model
    (eval_utils.py:1244-1420), composed here from the same reference metric calls in the
    same order, because that function itself only runs on trained-model folders on disk.
Only data is written: arrays, and JSON strings of the returned dicts (floats by repr, so
values round-trip exactly; NaN / Infinity allowed).
"""
import contextlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.ref_import import import_reference  # noqa: E402

import_reference()
import importlib  # noqa: E402

metrics = importlib.import_module("general_utils.metrics")
misc = importlib.import_module("general_utils.misc")
eu = importlib.import_module("evaluate.eval_utils")


def _j(obj):
    def conv(v):
        if v is None:
            return None
        if isinstance(v, dict):
            return dict((k, conv(x)) for k, x in v.items())
        if isinstance(v, (list, tuple)):
            return [conv(x) for x in v]
        return float(v)
    return json.dumps(conv(obj))


def quiet(fn, *a, **kw):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **kw)


def graphs(rng, p, L, n, density=0.3, quant=None):
    out = []
    for _ in range(n):
        g = rng.rand(p, p, L) * (rng.rand(p, p, 1) < density + 0.4)
        if quant:
            g = np.round(g * quant) / quant
        out.append(g)
    return out


def truths(rng, p, Lt, n, density=0.25):
    out = []
    for _ in range(n):
        t = np.zeros((p, p, Lt))
        t[..., 0] = (rng.rand(p, p) < density) * 1.0
        t[np.arange(p), np.arange(p), 0] = 1.0
        out.append(t)
    return out


def main():
    rng = np.random.RandomState(7)
    out = {}
    # --- per-graph scoring: flattened (score, label) pairs --------------------------------
    pairs = []
    for c in range(24):
        M = [100, 100, 64, 9][c % 4]
        s = rng.rand(M)
        if c % 3 == 0:
            s = np.round(s * 8) / 8          # many ties
        if c % 5 == 0:
            s[: M // 3] = 0.0                # block of zeros
        y = (rng.rand(M) < [0.3, 0.5, 0.1, 0.6][c % 4]).astype(np.int64)
        y[0], y[1] = 1, 0
        pairs.append((s, y))
    for c, (s, y) in enumerate(pairs):
        k = "pair%02d" % c
        out[k + "/score"], out[k + "/label"] = s, y
        thr, f1 = metrics.compute_optimal_f1(list(y), s)
        out[k + "/opt"] = np.array([thr, f1])
        res = {}
        for pc in (0.3, 0.5, 0.7, 0.9):
            res["f1_%s" % pc] = metrics.compute_f1(list(y), s, pc)
            with np.errstate(all="ignore"):
                res["sens_%s" % pc] = metrics.compute_sensitivity(list(y), s, pred_cutoff=pc)
                res["spec_%s" % pc] = metrics.compute_specificity(list(y), s, pred_cutoff=pc)
                res["plr_%s" % pc] = metrics.compute_positive_likelihood_ratio(list(y), s, pred_cutoff=pc)
                res["nlr_%s" % pc] = metrics.compute_negative_likelihood_ratio(list(y), s, pred_cutoff=pc)
        out[k + "/cutoffs"] = _j(res)
    # --- graph-level stats dicts (eval_utils.py:656-746), incl. edge cases ----------------
    cases = []
    for c in range(10):
        est = graphs(rng, 10, 4, 1, quant=(6 if c % 2 else None))[0].sum(axis=2)
        est = est / est.max()
        tru = truths(rng, 10, 2, 1)[0].sum(axis=2)
        cases.append((est, tru))
    cases.append((np.ones((10, 10)), truths(rng, 10, 2, 1)[0].sum(axis=2)))          # homogeneous est
    cases.append((rng.rand(10, 10), np.ones((10, 10))))                               # homogeneous labels
    bad = rng.rand(10, 10)
    bad[3, 4] = np.nan
    cases.append((bad, truths(rng, 10, 2, 1)[0].sum(axis=2)))                         # non-finite est
    for c, (est, tru) in enumerate(cases):
        k = "graph%02d" % c
        out[k + "/est"], out[k + "/true"] = est, tru
        with np.errstate(all="ignore"):
            out[k + "/optf1"] = _j(quiet(eu.compute_OptimalF1_stats_betw_two_gc_graphs, est, tru))
            out[k + "/f1s"] = _j(quiet(eu.compute_f1_stats_betw_two_gc_graphs, est, tru))
            out[k + "/key"] = _j(quiet(eu.compute_key_stats_betw_two_gc_graphs, est, tru))
        out[k + "/dc0"] = np.array([metrics.deltacon0(tru, est, 0.1, make_graphs_undirected=False),
                                    metrics.deltacon0(tru, est, 0.1, make_graphs_undirected=True)])
    # --- system-level factor statistics on model-like estimate sets ------------------------
    for c, (K, Lt, sort, excl, start) in enumerate([(4, 2, False, False, 0), (4, 4, True, False, 0),
                                                    (4, 4, True, True, 1), (3, 4, True, False, 0)]):
        k = "system%d" % c
        ests = graphs(rng, 10, 4, K, quant=(5 if c == 3 else None))
        trus = truths(rng, 10, Lt, K)
        out[k + "/meta"] = json.dumps(dict(K=K, sort=sort, exclude_self=excl, start=start))
        for i in range(K):
            out[k + "/est%d" % i], out[k + "/true%d" % i] = ests[i], trus[i]
        combo_e, combo_t = eu.get_combined_gc_representations_across_factors(ests, trus)
        out[k + "/combo_est"], out[k + "/combo_true"] = combo_e, combo_t
        cur = list(ests)
        if sort:
            cur, ei, gi = quiet(misc.sort_unsupervised_estimates, cur, trus, cost_criteria="CosineSimilarity",
                                unsupervised_start_index=start, return_sorting_inds=True)
            out[k + "/sort_inds"] = np.stack([np.asarray(ei), np.asarray(gi)])
        if excl:
            cur = [(1. - np.expand_dims(np.eye(x.shape[0]), 2)) * x for x in cur]
        cur = [x / np.max(x) for x in cur]
        stats = dict()
        for i, (tg, ge) in enumerate(zip(trus, cur)):
            tg = tg.sum(axis=2)
            ge = ge.sum(axis=2)
            lab = [int(v) for v in (1. * (tg > 0.)).flatten()]
            for T, e in (("", ge), ("T_", ge.T)):
                stats.setdefault(T + "cos_sim", []).append(metrics.compute_cosine_similarity(tg, e))
                stats.setdefault(T + "mse", []).append(metrics.compute_mse(tg, e))
                stats.setdefault(T + "dir_deltacon0", []).append(metrics.deltacon0(tg, e, 0.1, make_graphs_undirected=False))
                stats.setdefault(T + "undir_deltacon0", []).append(metrics.deltacon0(tg, e, 0.1, make_graphs_undirected=True))
                stats.setdefault(T + "deltacon0_wDD", []).append(metrics.deltacon0_with_directed_degrees(tg, e, 0.1, in_degree_coeff=1., out_degree_coeff=1.))
                stats.setdefault(T + "deltaffinity", []).append(metrics.deltaffinity(tg, e, 0.1, max_path_length=None))
                stats.setdefault(T + "roc_auc", []).append(eu.roc_auc_score(lab, e.flatten()))
            stats.setdefault("optf1", []).append(quiet(eu.compute_OptimalF1_stats_betw_two_gc_graphs, ge, 1. * (tg > 0.)))
        out[k + "/stats"] = _j(stats)
    np.savez_compressed(os.path.join(HERE, "eval_pipeline.npz"), **out)
    print("wrote eval_pipeline.npz (%d arrays)" % len(out))


if __name__ == "__main__":
    main()
