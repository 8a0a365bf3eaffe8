"""Host logic (CPU): the packed grid search's vectorised GC-progress / confusion trackers
(fit_loop.gc_progress_many, train_confusion_many) append exactly the values, in exactly the
histories, that the per-fit FitTracker methods (metrics.track_*_from_values, track_l1_stats,
track_cosine_stats_batched; model_utils.py:18-209) append -- bit for bit, including the
reference's length rules (one true graph for several supervised factors)."""
import copy
import types

import numpy as np
import pytest

from redcliff_amd import fit_loop
from redcliff_amd import metrics as M


def _tracker(p, K, nsup, GC):
    m = types.SimpleNamespace(num_supervised_factors=nsup, num_factors_nK=K, num_chans=p)
    return fit_loop.FitTracker(m, GC, 0.1, 1., 1., 1., 1., 1., 5, 1)


def _state(t):
    return {k: copy.deepcopy(getattr(t, k)) for k in ("f1_hist", "f1_off", "roc_hist", "roc_off", "l1_hist", "cos_hist",
                                                       "cos_unsup", "dc_hist", "dcdd_hist", "daff_hist", "plm_hist",
                                                       "cm_train")}


def _same(a, b):
    if isinstance(a, dict):
        return a.keys() == b.keys() and all(_same(a[k], b[k]) for k in a)
    if isinstance(a, list):
        return len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    if isinstance(a, np.ndarray):
        return np.array_equal(a, b, equal_nan=True) and a.dtype == b.dtype
    return (a == b and type(a) is type(b)) or (a != a and b != b)


@pytest.mark.parametrize("p,K,nsup,nG,S,Sn,ls", [(10, 4, 4, 4, 4, 40, 4), (6, 3, 2, 3, 2, 17, 3), (5, 3, 3, 1, 3, 9, 2),
                                                   (64, 8, 8, 8, 8, 40, 20), (7, 4, 1, 4, 1, 5, 1), (8, 5, 3, 3, 3, 12, 5)])
def test_gc_progress_many_bitwise(p, K, nsup, nG, S, Sn, ls):
    rng = np.random.RandomState(p * 100 + K)
    GC = [(rng.rand(p, p, ls) < 0.3).astype(np.float64) for _ in range(nG)]
    Ra, epochs = 3, 3
    solo = [_tracker(p, K, nsup, GC) for _ in range(Ra)]
    many = [_tracker(p, K, nsup, GC) for _ in range(Ra)]
    G = min(K, nG)
    for _ in range(epochs):
        est = rng.rand(Ra, S, K, p, p, ls).astype(np.float32) * rng.choice([1e-3, 1.0, 1e3])
        est[rng.rand(*est.shape) < 0.2] = 0.0
        nolag = (rng.rand(Ra, Sn, K, p, p, 1).astype(np.float32) - 0.1)
        vals = rng.randn(Ra, S, G, 6 + p)
        for i, t in enumerate(solo):
            est_np = [[est[i, s, k] for k in range(K)] for s in range(S)]
            t.gc_progress(est_np, nolag[i], vals[i])
        fit_loop.gc_progress_many(many, vals, *M.track_values_host(est, nolag))
        cms = rng.randint(0, 50, size=(Ra, max(nsup, 1), max(nsup, 1)))
        cms[0, 0] = 0  # an empty class: nan rates
        for i, t in enumerate(solo):
            t.train_confusion(cms[i] if nsup > 0 else None)
        fit_loop.train_confusion_many(many, cms)
    for a, b in zip(solo, many):
        sa, sb = _state(a), _state(b)
        assert all(len(h) == epochs for h in sa["l1_hist"]) and all(len(h) == epochs for h in sa["dc_hist"])
        assert all(len(h) == epochs for h in sa["cos_hist"].values())
        for k in sa:
            assert _same(sa[k], sb[k]), k


@pytest.mark.parametrize("with_cols", [False, True])
@pytest.mark.parametrize("p,K,nsup,nG,S,Sn,ls", [(10, 4, 4, 4, 4, 40, 4), (5, 3, 3, 1, 3, 9, 2), (8, 5, 3, 3, 3, 12, 5)])
def test_deferred_histories_bitwise(p, K, nsup, nG, S, Sn, ls, with_cols):
    """DeferredHistories (the packed fit's per-epoch log, flushed before checkpoints and at the
    end) appends the same values, in the same order, as the per-epoch appends -- with replicas
    leaving the active set (early stopping) and a flush in the middle (a checkpoint epoch)."""
    rng = np.random.RandomState(7 * p + K)
    GC = [(rng.rand(p, p, ls) < 0.3).astype(np.float64) for _ in range(nG)]
    R, epochs = 4, 6
    now = [_tracker(p, K, nsup, GC) for _ in range(R)]
    lazy = [_tracker(p, K, nsup, GC) for _ in range(R)]
    log = fit_loop.DeferredHistories()
    G = min(K, nG)
    active = list(range(R))
    for e in range(epochs):
        Ra = len(active)
        est = rng.rand(Ra, S, K, p, p, ls).astype(np.float32)
        nolag = (rng.rand(Ra, Sn, K, p, p, 1).astype(np.float32) - 0.1)
        vals = rng.randn(Ra, S, G, 6 + p)
        stats = M.track_values_host(est, nolag)
        fit_loop.gc_progress_many([now[r] for r in active], vals, *stats)
        cols = active if with_cols else None  # the pack passes its replica indices
        fit_loop.gc_progress_many([lazy[r] for r in active], vals, *stats, log=log, cols=cols)
        cms = rng.randint(0, 50, size=(Ra, max(nsup, 1), max(nsup, 1)))
        fit_loop.train_confusion_many([now[r] for r in active], cms)
        fit_loop.train_confusion_many([lazy[r] for r in active], cms, log=log, cols=cols)
        # the cosine histories (the stopping rule reads them) are appended at once
        for r in active:
            assert _same(now[r].cos_hist, lazy[r].cos_hist)
        if e == 2:
            log.flush()
            for a, b in zip(now, lazy):
                assert _same(_state(a), _state(b))
        if e == 1:
            active = [0, 1, 3]  # replica 2 stopped at epoch 1
        if e == 3:
            active = [1, 3]
    log.flush()
    for a, b in zip(now, lazy):
        sa, sb = _state(a), _state(b)
        for k in sa:
            assert _same(sa[k], sb[k]), k
    assert len(now[2].l1_hist[0]) == 2 and len(now[1].l1_hist[0]) == epochs
