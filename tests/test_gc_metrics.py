"""Per-epoch GC-progress metrics of fit() (general_utils/model_utils.py:18-209 over
general_utils/metrics.py) against the reference's own trackers run on seeded estimates
(tests/golden/gc_metrics.npz, written by tests/golden/make_golden.py run_metrics):
  * host restatement (redcliff_amd.metrics, CPU);
  * GPU kernel rc_metrics.hip through redcliff_gc_progress (-m gpu).
Tolerances: F1 and ROC-AUC (counts, float32 F1 arithmetic) to 1e-12; the continuous
metrics to 1e-6 relative (float32 matrix powers and LAPACK's LU vs Gauss-Jordan round
differently); NaN where the reference gives NaN."""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))

D = np.load(os.path.join(HERE, "golden", "gc_metrics.npz"))
CASES = sorted(set(k.split("/")[0] for k in D.files))


def case(name):
    meta = json.loads(str(D[name + "/meta"]))
    return meta, dict((k.split("/", 1)[1], D[k]) for k in D.files if k.startswith(name + "/"))


def close(tag, got, want, rtol, atol=0.0):
    got, want = np.asarray(got, dtype=np.float64), np.asarray(want, dtype=np.float64)
    assert got.shape == want.shape, (tag, got.shape, want.shape)
    assert np.array_equal(np.isnan(got), np.isnan(want)), (tag, got, want)
    m = ~np.isnan(want)
    np.testing.assert_allclose(got[m], want[m], rtol=rtol, atol=atol, err_msg=tag)


def _hists(nsup, p):
    return ({0.0: [[] for _ in range(nsup)]}, {0.0: [[] for _ in range(nsup)]}, {0.0: [[] for _ in range(nsup)]},
            {0.0: [[] for _ in range(nsup)]}, [[] for _ in range(nsup)], [[] for _ in range(nsup)],
            [[] for _ in range(nsup)], {pl: [[] for _ in range(nsup)] for pl in range(1, p)})


def _check(name, meta, d, f1, roc, f1o, roco, dc, dcdd, daff, plm, rt):
    nsup, p = meta["nsup"], meta["p"]
    close(name + " f1", [h[0] for h in f1[0.0]], d["f1"], 1e-12, 1e-12)
    close(name + " roc", [h[0] for h in roc[0.0]], d["roc"], 1e-12, 1e-12)
    close(name + " f1_off", [h[0] for h in f1o[0.0]], d["f1_off"], 1e-12, 1e-12)
    close(name + " roc_off", [h[0] for h in roco[0.0]], d["roc_off"], 1e-12, 1e-12)
    close(name + " dc", [h[0] for h in dc], d["dc"], rt)
    close(name + " dcdd", [h[0] for h in dcdd], d["dcdd"], rt)
    close(name + " daff", [h[0] for h in daff], d["daff"], rt)
    got = np.asarray([[plm[pl][i][0] if plm[pl][i] else np.nan for i in range(nsup)] for pl in range(1, p)])
    close(name + " plm", got, d["plm"], rt)


@pytest.mark.parametrize("name", CASES)
def test_host_metrics_match_reference(name):
    from redcliff_amd import metrics as M
    meta, d = case(name)
    S, K, nsup, p = meta["S"], meta["K"], meta["nsup"], meta["p"]
    est = [[d["est"][s, k] for k in range(K)] for s in range(S)]
    GC = [d["gc"][g] for g in range(meta["G"])]
    f1, roc, f1o, roco, dc, dcdd, daff, plm = _hists(nsup, p)
    with np.errstate(all="ignore"):
        M.track_roc_stats(GC, est, f1, roc, False)
        M.track_roc_stats(GC, est, f1o, roco, True)
        M.track_deltacon_stats(GC, est, p, dc, dcdd, daff, plm, 0.1, 1., 0.5)
    _check(name, meta, d, f1, roc, f1o, roco, dc, dcdd, daff, plm, 1e-6)
    l1 = [[] for _ in range(nsup)]
    M.track_l1_stats(est, l1)
    close(name + " l1", [h[0] for h in l1], d["l1"], 1e-6)
    cos = {"%dand%d" % (i, j): [] for i in range(K) for j in range(K) if i < j}
    M.track_cosine_stats_batched(d["nolag"], cos)
    close(name + " cos", [cos[k][0] for k in sorted(cos)], d["cos"], 1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_device_metrics_match_reference(name):
    import torch
    from redcliff_amd import metrics as M
    meta, d = case(name)
    nsup, p = meta["nsup"], meta["p"]
    GC = [d["gc"][g] for g in range(meta["G"])]
    vals = M.gc_progress_values(GC, torch.from_numpy(d["est"]).cuda(), 0.1, 1., 0.5)
    f1, roc, f1o, roco, dc, dcdd, daff, plm = _hists(nsup, p)
    M.track_roc_stats_from_values(vals, f1, roc, False)
    M.track_roc_stats_from_values(vals, f1o, roco, True)
    M.track_deltacon_stats_from_values(vals, p, dc, dcdd, daff, plm)
    _check(name, meta, d, f1, roc, f1o, roco, dc, dcdd, daff, plm, 1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("p,L,S,K", [(10, 4, 4, 4), (12, 20, 3, 9), (64, 20, 2, 8), (33, 8, 2, 3)])
def test_device_metrics_match_host_restatement(p, L, S, K):
    """Shapes beyond the fixtures (up to the stress config's p=64 and 20 lags): device vs the
    host restatement that the fixtures pin."""
    import torch
    from redcliff_amd import metrics as M
    rng = np.random.RandomState(p * 100 + L)
    est = (rng.rand(S, K, p, p, L) - 0.1).astype(np.float32) / np.float32(p)
    gc = [(rng.rand(p, p, 2) > 0.8).astype(np.float64) for _ in range(K)]
    vals = M.gc_progress_values(gc, torch.from_numpy(est).cuda(), 0.1, 1., 1.)
    f1, roc, f1o, roco, dc, dcdd, daff, plm = _hists(K, p)
    M.track_roc_stats_from_values(vals, f1, roc, False)
    M.track_roc_stats_from_values(vals, f1o, roco, True)
    M.track_deltacon_stats_from_values(vals, p, dc, dcdd, daff, plm)
    h = _hists(K, p)
    estl = [[est[s, k] for k in range(K)] for s in range(S)]
    with np.errstate(all="ignore"):
        M.track_roc_stats(gc, estl, h[0], h[1], False)
        M.track_roc_stats(gc, estl, h[2], h[3], True)
        M.track_deltacon_stats(gc, estl, p, h[4], h[5], h[6], h[7], 0.1, 1., 1.)
    want = dict(f1=[x[0] for x in h[0][0.0]], roc=[x[0] for x in h[1][0.0]], f1_off=[x[0] for x in h[2][0.0]],
                roc_off=[x[0] for x in h[3][0.0]], dc=[x[0] for x in h[4]], dcdd=[x[0] for x in h[5]],
                daff=[x[0] for x in h[6]],
                plm=np.asarray([[h[7][pl][i][0] for i in range(K)] for pl in range(1, p)]))
    _check("p%d" % p, dict(nsup=K, p=p), want, f1, roc, f1o, roco, dc, dcdd, daff, plm, 1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("p,L,S,Sn,K,R", [(10, 4, 4, 40, 4, 3), (64, 20, 8, 40, 8, 1), (7, 3, 2, 5, 5, 2)])
def test_device_tracker_stats_match_host(p, L, S, Sn, K, R):
    """redcliff_gc_track_stats (per-estimate L1 values, normalised dot products of the lag-free
    estimates; model_utils.py:163-209) vs the trackers' numpy reductions: the device sums in its
    own fixed order, so 1e-12 relative; and the values of one replica do not depend on the
    number of replicas in the launch (bitwise)."""
    import torch
    from redcliff_amd import metrics as M
    rng = np.random.RandomState(p + L)
    est = (rng.rand(R, S, K, p, p, L) - 0.05).astype(np.float32)
    nolag = (rng.rand(R, Sn, K, p, p, 1) - 0.05).astype(np.float32)
    got = M.gc_track_values(torch.from_numpy(est).cuda(), torch.from_numpy(nolag).cuda())
    want = M.track_values_host(est, nolag)
    for tag, g, w in zip(("l1", "nrm", "dots"), got, want):
        if tag == "dots":
            iu = np.triu_indices(K)
            g, w = g[..., iu[0], iu[1]], w[..., iu[0], iu[1]]
        np.testing.assert_allclose(g, w, rtol=1e-12, atol=0, err_msg=tag)
    one = M.gc_track_values(torch.from_numpy(est[-1:]).cuda(), torch.from_numpy(nolag[-1:]).cuda())
    for g, o in zip(got, one):
        assert np.array_equal(g[-1:], o)
