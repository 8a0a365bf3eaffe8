"""Packed grid-search fit (ReplicaPack.fit, the fits/hour unit of BASELINE.metric) against R
independent fit() calls (models/redcliff_s_cmlp_withStateSmoothing.py:1175-1647, one SLURM task
per grid point in the reference, train/REDCLIFF_S_CMLP_tst100hzRerun1024AvgReg_gsSmooth1.py:
125-160).  Every replica must end bit-identical to its independent fit -- parameters, BatchNorm
buffers, loss histories, best epoch, the epoch it stopped at -- including replicas that stop
at different epochs (a stopped replica leaves the launch's active list)."""
import os

import numpy as np
import pytest
import torch

from test_gpu_replicas import data, make, opts

pytestmark = pytest.mark.gpu

# (seed, FORECAST_COEFF, ADJ_L1 scale, gen_lr, embed_lr, stopping forecast coeff, stopping factor coeff)
GRID = [
    (0, 10.0, 0.1, 5e-4, 2e-4, 10.0, 100.0),
    (1, 1.0, 0.01, 1e-3, 1e-3, 1.0, 100.0),
    (2, 10.0, 0.01, 5e-4, 1e-4, 10.0, 1.0),
    (3, 1.0, 0.1, 2e-3, 5e-4, 10.0, 10.0),
]
HKEYS = ("avg_forecasting_loss", "avg_factor_loss", "avg_factor_cos_sim_penalty", "avg_fw_l1_penalty",
         "avg_adj_penalty", "avg_combo_loss")


def same(a, b):
    """Bitwise equality of nested history containers; NaN equals NaN (deltacon0 of a graph whose
    similarity matrix has negative entries is NaN in the reference too, general_utils/metrics.py)."""
    if isinstance(a, dict):
        return isinstance(b, dict) and a.keys() == b.keys() and all(same(a[k], b[k]) for k in a)
    if isinstance(a, (list, tuple)):
        return isinstance(b, (list, tuple)) and len(a) == len(b) and all(same(x, y) for x, y in zip(a, b))
    if isinstance(a, (float, np.floating)) and isinstance(b, (float, np.floating)):
        return (np.isnan(a) and np.isnan(b)) or a == b
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        return np.array_equal(np.asarray(a), np.asarray(b), equal_nan=True)
    return a == b


def true_graphs(K, p, L, seed=11):
    rng = np.random.RandomState(seed)
    return [(rng.rand(p, p, L) < 0.3).astype(np.float64) for _ in range(K)]


@pytest.mark.parametrize("path,save", [("vector", True), ("mfma", True), ("vector", False), ("mfma", False)])
def test_pack_fit_bitwise_equals_independent_fits(path, save, monkeypatch, tmp_path):
    """save=False: no checkpoint files, so every epoch but the last trains the next one
    speculatively while the host digests the current one, and replicas that stop are rolled
    back (ReplicaPack._roll_back); their Adam moments and step counts are compared too."""
    from redcliff_amd import ReplicaPack
    monkeypatch.setenv("REDCLIFF_FAC_PATH", path)
    train = data(64 * 2 + 24, seed=3)
    val = data(96, seed=4)
    gc = true_graphs(4, 10, 4)
    kw = dict(lookback=1, check_every=1, GC=gc, deltaConEps=0.1)
    max_iter = 9
    solo, solo_opts = [], []
    for s, fc, adj, lrB, lrA, scf, scfa in GRID:
        m = make(s, fc, adj)
        oA, oB = opts(m, lrB, lrA)
        solo_opts.append((oA, oB))
        m.fit(None, train, oA, oB, 4, 1, 1, max_iter, val, verbose=0, stopping_criteria_forecast_coeff=scf,
              stopping_criteria_factor_coeff=scfa, stopping_criteria_cosSim_coeff=1., **kw)
        torch.cuda.synchronize()
        solo.append(m)
    packed = [make(s, fc, adj) for s, fc, adj, _, _, _, _ in GRID]
    pack_opts = [opts(m, lrB, lrA) for m, (_, _, _, lrB, lrA, _, _) in zip(packed, GRID)]
    pack = ReplicaPack(packed, pack_opts)
    finals = pack.fit(str(tmp_path) if save else None, train, val, max_iter, verbose=0,
                      stopping_criteria_forecast_coeff=[g[5] for g in GRID],
                      stopping_criteria_factor_coeff=[g[6] for g in GRID], stopping_criteria_cosSim_coeff=1., **kw)
    torch.cuda.synchronize()
    stops = []
    for r, (a, b) in enumerate(zip(solo, packed)):
        ha, hb = a.fit_history, b.fit_history
        assert hb["best_it"] == ha["best_it"], r
        assert hb["stopped_at"] == ha["stopped_at"], r
        stops.append(ha["stopped_at"])
        for k in HKEYS:
            assert same(hb[k], ha[k]), "replica %d %s" % (r, k)
        for k in ("f1score_histories", "roc_auc_histories", "deltacon0_histories"):
            assert same(hb[k], ha[k]), "replica %d %s" % (r, k)
        sa, sb = a.state_dict(), b.state_dict()
        for k in sa:
            np.testing.assert_array_equal(sb[k].cpu().numpy(), sa[k].cpu().numpy(), err_msg="replica %d %s" % (r, k))
        for oa, ob in zip(solo_opts[r], pack_opts[r]):
            stA, stB = oa.state_dict()["state"], ob.state_dict()["state"]
            assert stA.keys() == stB.keys()
            for i in stA:
                for k in ("exp_avg", "exp_avg_sq", "step"):
                    np.testing.assert_array_equal(stB[i][k].cpu().numpy(), stA[i][k].cpu().numpy(),
                                                  err_msg="replica %d optimizer state %s %s" % (r, i, k))
        if save:  # the final model file holds this replica's own parameters only
            f = os.path.join(str(tmp_path), "replica_%d" % r, "final_best_model.bin")
            nparam = sum(t.numel() for t in b.parameters())
            assert os.path.getsize(f) < 4 * nparam * 1.5 + 2 ** 20
    assert len(finals) == len(GRID)
    print("stop epochs:", stops)
    assert any(s is not None for s in stops), "no replica stopped early: the active-list path went untested"


# (pretrain epochs, acclimation epochs) per replica: the TST grid's schedule axes
# (train/REDCLIFF_S_CMLP_tst100hzRerun1024AvgReg_gsSmooth1.py:297-298), scaled down
SCHEDULES = [(1, 1), (2, 1), (1, 3), (3, 2)]


@pytest.mark.parametrize("path", ["vector", "mfma"])
def test_mixed_schedule_per_replica_data_pack_fit_bitwise(path, monkeypatch):
    """The reference's real grids in one pack: every replica has its own phase schedule (the pack
    launches one chain per phase group each epoch; Adam step numbers per replica through the hyper
    rows' t_offset) and its own training / validation data and true graphs (PerReplica: the
    synthetic grid's one-model-many-datasets form, ...BSCgsSmooth3Parsim.py:66-72).  Every replica
    ends bit-identical to its independent fit(), histories, stopping epoch and Adam state
    included."""
    from redcliff_amd import PerReplica, ReplicaPack
    monkeypatch.setenv("REDCLIFF_FAC_PATH", path)
    trains = [data(64 * 2 + 24, seed=30 + r) for r in range(len(GRID))]
    vals = [data(96, seed=40 + r) for r in range(len(GRID))]
    gcs = [true_graphs(4, 10, 4, seed=50 + r) for r in range(len(GRID))]
    max_iter = 10
    kw = dict(lookback=1, check_every=1, deltaConEps=0.1)
    solo, solo_opts = [], []
    for r, (s, fc, adj, lrB, lrA, scf, scfa) in enumerate(GRID):
        pre, acc = SCHEDULES[r]
        m = make(s, fc, adj, pre=pre, acc=acc)
        oA, oB = opts(m, lrB, lrA)
        solo_opts.append((oA, oB))
        m.fit(None, trains[r], oA, oB, 4, 1, 1, max_iter, vals[r], verbose=0, GC=gcs[r],
              stopping_criteria_forecast_coeff=scf, stopping_criteria_factor_coeff=scfa,
              stopping_criteria_cosSim_coeff=1., **kw)
        torch.cuda.synchronize()
        solo.append(m)
    packed = [make(g[0], g[1], g[2], pre=SCHEDULES[r][0], acc=SCHEDULES[r][1]) for r, g in enumerate(GRID)]
    pack_opts = [opts(m, g[3], g[4]) for m, g in zip(packed, GRID)]
    pack = ReplicaPack(packed, pack_opts)
    # epoch 1: replicas 0 and 2 acclimate while 1 and 3 still pretrain the embedder
    assert len(pack.phase_groups(1)) == 2
    pack.fit(None, PerReplica(trains), PerReplica(vals), max_iter, verbose=0, GC=PerReplica(gcs),
             stopping_criteria_forecast_coeff=[g[5] for g in GRID], stopping_criteria_factor_coeff=[g[6] for g in GRID],
             stopping_criteria_cosSim_coeff=1., **kw)
    torch.cuda.synchronize()
    for r, (a, b) in enumerate(zip(solo, packed)):
        ha, hb = a.fit_history, b.fit_history
        assert hb["best_it"] == ha["best_it"] and hb["stopped_at"] == ha["stopped_at"], r
        for k in HKEYS + ("f1score_histories", "roc_auc_histories", "deltacon0_histories",
                          "gc_factor_cosine_sim_histories"):
            assert same(hb[k], ha[k]), "replica %d %s" % (r, k)
        sa, sb = a.state_dict(), b.state_dict()
        for k in sa:
            np.testing.assert_array_equal(sb[k].cpu().numpy(), sa[k].cpu().numpy(), err_msg="replica %d %s" % (r, k))
        for oa, ob in zip(solo_opts[r], pack_opts[r]):
            stA, stB = oa.state_dict()["state"], ob.state_dict()["state"]
            for i in stA:
                for k in ("exp_avg", "exp_avg_sq", "step"):
                    np.testing.assert_array_equal(stB[i][k].cpu().numpy(), stA[i][k].cpu().numpy(),
                                                  err_msg="replica %d optimizer state %s %s" % (r, i, k))


def test_fit_packs_interleaved_equals_pack_fits(monkeypatch):
    """fit_packs: two packs of different shapes (K = 4 and K = 3 factors: two shape classes of the
    synthetic grid) fitted concurrently, one stream each, every epoch of both enqueued before the host
    waits -- each replica bit-identical to its pack fitted alone."""
    import redcliff_amd
    from redcliff_amd import ReplicaPack, fit_packs
    import test_gpu_replicas as T
    monkeypatch.setenv("REDCLIFF_FAC_PATH", "mfma")
    train, val = data(64 * 2 + 24, seed=61), data(96, seed=62)
    gc4 = true_graphs(4, 10, 4, seed=63)
    kw = dict(lookback=1, check_every=1, deltaConEps=0.1, verbose=0, stopping_criteria_forecast_coeff=10.,
              stopping_criteria_factor_coeff=100., stopping_criteria_cosSim_coeff=1.)

    def packs():
        a = [make(s, fc, adj) for s, fc, adj, _, _, _, _ in GRID]
        oa = [opts(m, g[3], g[4]) for m, g in zip(a, GRID)]
        saved = dict(T.CFG)
        T.CFG.update(K=3, nsup=3)
        try:
            b = [make(10 + s, fc, adj) for s, fc, adj, _, _, _, _ in GRID[:3]]
        finally:
            T.CFG.clear()
            T.CFG.update(saved)
        ob = [opts(m, g[3], g[4]) for m, g in zip(b, GRID)]
        return (ReplicaPack(a, oa), a), (ReplicaPack(b, ob), b)
    Y3 = [(X, Yb[:, :3]) for X, Yb in train]
    V3 = [(X, Yb[:, :3]) for X, Yb in val]
    gc3 = gc4[:3]
    (pa, ma), (pb, mb) = packs()
    pa.fit(None, train, val, 8, GC=gc4, **kw)
    pb.fit(None, Y3, V3, 8, GC=gc3, **kw)
    torch.cuda.synchronize()
    (qa, na), (qb, nb) = packs()
    fit_packs([(qa, (None, train, val, 8), dict(GC=gc4, **kw)), (qb, (None, Y3, V3, 8), dict(GC=gc3, **kw))])
    torch.cuda.synchronize()
    for x, y in list(zip(ma, na)) + list(zip(mb, nb)):
        assert x.fit_history["best_it"] == y.fit_history["best_it"]
        assert same(x.fit_history["avg_combo_loss"], y.fit_history["avg_combo_loss"])
        sa, sb = x.state_dict(), y.state_dict()
        for k in sa:
            np.testing.assert_array_equal(sb[k].cpu().numpy(), sa[k].cpu().numpy(), err_msg=k)


@pytest.mark.parametrize("K,p", [(1, 3), (2, 3), (1, 12), (10, 6)])
@pytest.mark.parametrize("kern", ["vector", "mfma-gemm"])
def test_synthetic_grid_shape_classes_pack_fit(K, p, kern, monkeypatch):
    """Shape classes of the reference's synthetic grid (num_factors = num_supervised_factors = numF in
    1..10, numN in {3, 6, 12}, train/REDCLIFF_S_CMLP_synSysInnovGauss1030_BSCgsSmooth3Parsim.py:97-100,
    140-1131; model: h = 25, gen_lag 4, DGCNN 16 / 3 / 100) as PerReplica packs -- the extremes a GPU's
    share can hold (a single factor, three channels) -- each replica bit-identical to its own fit().
    kern "mfma-gemm": the packed grids' kernels (short-contraction factor kernels, GEMM-shaped embedder)."""
    import redcliff_amd
    monkeypatch.setenv("REDCLIFF_FAC_PATH", "vector" if kern == "vector" else "mfma")
    if kern != "vector":
        monkeypatch.setenv("REDCLIFF_EMB_PATH", "gemm")
    from redcliff_amd import PerReplica, ReplicaPack

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
    solo = []
    for r in range(R):
        m = model(100 + r)
        oA, oB = opts(m, 5e-4, 5e-4)
        m.fit(None, trains[r], oA, oB, 4, 1, 1, 7, vals[r], GC=gcs[r], **kw)
        solo.append(m)
    packed = [model(100 + r) for r in range(R)]
    pack = ReplicaPack(packed, [opts(m, 5e-4, 5e-4) for m in packed])
    pack.fit(None, PerReplica(trains), PerReplica(vals), 7, GC=PerReplica(gcs), **kw)
    torch.cuda.synchronize()
    for r, (a, b) in enumerate(zip(solo, packed)):
        assert b.fit_history["best_it"] == a.fit_history["best_it"], r
        for k in HKEYS:
            assert same(b.fit_history[k], a.fit_history[k]), "replica %d %s" % (r, k)
        sa, sb = a.state_dict(), b.state_dict()
        for k in sa:
            np.testing.assert_array_equal(sb[k].cpu().numpy(), sa[k].cpu().numpy(), err_msg="replica %d %s" % (r, k))
