"""Grid-search replicas packed into one launch (redcliff_amd.ReplicaPack)
must reproduce R independent fits exactly: same kernels, the replica only moves to
blockIdx.y, so parameters, BatchNorm buffers, Adam state and validation losses are
compared bit for bit against the same models stepped one at a time on the same factor path."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = dict(p=10, L=4, K=4, nsup=4, h=100, F=20, n=2, H=30, T=21)  # D4IC-shaped (BASELINE configs[1])
GRID = [  # (seed, FORECAST_COEFF, ADJ_L1 scale, gen_lr, embed_lr)
    (0, 10.0, 0.1, 5e-4, 2e-4),
    (1, 1.0, 0.01, 1e-4, 5e-4),
    (2, 10.0, 0.01, 5e-4, 1e-4),
]
# packs of >= 8 replicas take the packed-only code paths (8 windows per forward workgroup, one
# stream, the embedder-backward partials combined by the final kernel): 8 grid points
GRID8 = GRID + [(3 + i, (1.0, 10.0)[i % 2], (0.1, 0.01)[i % 2], (5e-4, 1e-4)[i % 2], (2e-4, 5e-4)[i % 2])
                for i in range(5)]


def make(seed, fc, adj, pre=1, acc=1, mode="pretrain_embedder_then_acclimate_factors_then_combined"):
    import redcliff_amd
    K, p = CFG["K"], CFG["p"]
    coeff = {"FORECAST_COEFF": fc, "FACTOR_SCORE_COEFF": 100.0, "FACTOR_COS_SIM_COEFF": 1.0 / sum(range(1, K)),
             "FACTOR_WEIGHT_L1_COEFF": 1e-3, "FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF": 0.0,
             "ADJ_L1_REG_COEFF": adj / K / np.sqrt(p * p - 1.0), "DAGNESS_REG_COEFF": 0.0, "DAGNESS_LAG_COEFF": 0.0,
             "DAGNESS_NODE_COEFF": 0.0}
    eargs = [("num_features_per_node", CFG["F"]), ("num_graph_conv_layers", CFG["n"]),
             ("num_hidden_nodes", CFG["H"]), ("sigmoid_eccentricity_coeff", 10.0)]
    torch.manual_seed(seed)
    return redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing(
        p, CFG["L"], [CFG["h"]], CFG["F"], [0], CFG["L"], 1, K, CFG["nsup"], coeff, False, "DGCNN", eargs,
        "conditional_factor_fixed_embedder", "apply_factor_weights_after_sim_completion", num_sims=1,
        training_mode=mode, num_pretrain_epochs=pre,
        num_acclimation_epochs=acc).cuda()


def opts(m, lrB, lrA):
    oA = torch.optim.Adam(m.gen_model[0].parameters(), lr=lrA, betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    oB = torch.optim.Adam(m.gen_model[1].parameters(), lr=lrB, betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    return oA, oB


def data(N, seed):
    rng = np.random.RandomState(seed)
    X = rng.randn(N, CFG["T"], CFG["p"]).astype(np.float32)
    Y = np.zeros((N, CFG["K"], 1), np.float32)
    Y[np.arange(N), rng.randint(0, CFG["K"], N), 0] = 10.0
    X, Y = torch.from_numpy(X), torch.from_numpy(Y)
    return [(X[i:i + 64], Y[i:i + 64]) for i in range(0, N, 64)]


@pytest.mark.parametrize("emb", [None, "gemm"])
def test_pack_xcd_orders_bitwise(emb, monkeypatch):
    """XCD-aware workgroup orders (rc_gemm_tile for the GEMM core, rc_xcd_order for k_fac_mix and the
    short-contraction factor kernels: every workgroup of one replica on one XCD once the replica
    count is a multiple of 8) against dispatch order (REDCLIFF_*_XCD=0): a bijection of the same
    workgroups, so 8 replicas trained through all three phases end bit-identical."""
    from redcliff_amd import ReplicaPack
    monkeypatch.setenv("REDCLIFF_FAC_PATH", "mfma")
    if emb:
        monkeypatch.setenv("REDCLIFF_EMB_PATH", emb)
    train = data(64 * 2 + 24, seed=9)
    states = {}
    for v in ("1", "0"):
        for k in ("REDCLIFF_GEMM_XCD", "REDCLIFF_MIX_XCD", "REDCLIFF_S16_XCD"):
            monkeypatch.setenv(k, v)
        models = [make(s, fc, adj) for s, fc, adj, _, _ in GRID8]
        pack = ReplicaPack(models, [opts(m, lrB, lrA) for m, (_, _, _, lrB, lrA) in zip(models, GRID8)])
        ds = pack.cache_dataset(train)
        for epoch in (0, 1, 2, 3):
            pack.run_epoch(epoch, ds)
        torch.cuda.synchronize()
        states[v] = [{k: t.detach().cpu().numpy() for k, t in m.state_dict().items()} for m in models]
    for r, (a, b) in enumerate(zip(states["1"], states["0"])):
        for k in a:
            np.testing.assert_array_equal(a[k], b[k], err_msg="replica %d %s" % (r, k))


@pytest.mark.parametrize("path,grid,emb", [("vector", GRID, None), ("mfma", GRID, None), ("mfma", GRID8, None),
                                          ("mfma", GRID, "gemm"), ("mfma", GRID8, "gemm")])
def test_packed_replicas_match_independent_fits(path, grid, emb, monkeypatch):
    """Both factor paths (the default picks the matrix cores for packs of >= 8 replicas, so the
    path is pinned here to compare like with like); R = 3 and the packed-only paths at R = 8.
    emb "gemm": the GEMM-shaped embedder with its products batched over the replicas, against
    single fits on the same embedder path (the default of packs of >= 16 replicas)."""
    monkeypatch.setenv("REDCLIFF_FAC_PATH", path)
    if emb:
        monkeypatch.setenv("REDCLIFF_EMB_PATH", emb)
    GRID = grid
    from redcliff_amd import ReplicaPack
    train = data(64 * 2 + 24, seed=3)  # two full batches + a ragged one
    val = data(80, seed=4)
    solo = [make(s, fc, adj) for s, fc, adj, _, _ in GRID]
    solo_opts = [opts(m, lrB, lrA) for m, (_, _, _, lrB, lrA) in zip(solo, GRID)]
    packed = [make(s, fc, adj) for s, fc, adj, _, _ in GRID]
    pack = ReplicaPack(packed, [opts(m, lrB, lrA) for m, (_, _, _, lrB, lrA) in zip(packed, GRID)])
    ds = pack.cache_dataset(train)
    vds = pack.cache_dataset(val)
    for epoch in (0, 1, 2, 3):  # pretrain-embedder, acclimate, combined, combined
        pack.run_epoch(epoch, ds)
        for m, (oA, oB) in zip(solo, solo_opts):
            for bi, (Xb, Yb) in enumerate(train):
                m.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
    torch.cuda.synchronize()
    losses, conf = pack.validate(vds)
    for r, (m, mp) in enumerate(zip(solo, packed)):
        a, b = m.state_dict(), mp.state_dict()
        assert set(a) == set(b)
        for k in a:
            np.testing.assert_array_equal(b[k].cpu().numpy(), a[k].cpu().numpy(), err_msg="replica %d %s" % (r, k))
        hist = [[] for _ in range(5)]
        v = m.validate_training(val, 1, CFG["p"], *hist)
        want = [v[0], v[1], v[2], v[3], v[4], v[5], v[9]]  # ..., adj, (3 DAG terms), combo
        np.testing.assert_allclose(losses[r], want, rtol=1e-6, atol=1e-9, err_msg="replica %d losses" % r)
    # the packed models remain ordinary drop-in modules afterwards
    Xv = val[0][0][:8, :CFG["F"]].cuda()
    solo[1].eval()
    packed[1].eval()
    with torch.no_grad():
        g1 = solo[1].GC("conditional_factor_fixed_embedder", X=Xv, threshold=False, ignore_lag=False)
        g2 = packed[1].GC("conditional_factor_fixed_embedder", X=Xv, threshold=False, ignore_lag=False)
    np.testing.assert_array_equal(g2[3][2].cpu().numpy(), g1[3][2].cpu().numpy())


@pytest.mark.parametrize("path,emb", [("vector", None), ("mfma", None), ("vector", "gemm"), ("mfma", "gemm")])
def test_single_active_replica_bitwise(path, emb, monkeypatch):
    """A pack whose active list has ONE entry that is not replica 0 (every other replica has stopped
    early): each launch then has one replica in its grid, and every kernel -- the GEMM core's
    replica axis included -- must still address that replica's parameters and workspace.  Replica 2
    trains alone for epochs 2 and 3 and ends bit-identical to its independent fit; the stopped
    replicas are left untouched."""
    monkeypatch.setenv("REDCLIFF_FAC_PATH", path)
    if emb:
        monkeypatch.setenv("REDCLIFF_EMB_PATH", emb)
    from redcliff_amd import ReplicaPack
    train = data(64 * 2 + 24, seed=13)
    val = data(80, seed=14)
    solo = make(*GRID[2][:3])
    oA, oB = opts(solo, GRID[2][3], GRID[2][4])
    packed = [make(s, fc, adj) for s, fc, adj, _, _ in GRID]
    pack = ReplicaPack(packed, [opts(m, lrB, lrA) for m, (_, _, _, lrB, lrA) in zip(packed, GRID)])
    ds = pack.cache_dataset(train)
    vds = pack.cache_dataset(val)
    for epoch in (0, 1, 2, 3):
        if epoch == 2:
            torch.cuda.synchronize()
            frozen = [{k: t.detach().cpu().numpy().copy() for k, t in m.state_dict().items()} for m in packed[:2]]
        pack.run_epoch(epoch, ds, active=None if epoch < 2 else [2])
        for bi, (Xb, Yb) in enumerate(train):
            solo.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
    torch.cuda.synchronize()
    losses, _ = pack.validate(vds, active=[2])
    a, b = solo.state_dict(), packed[2].state_dict()
    for k in a:
        np.testing.assert_array_equal(b[k].cpu().numpy(), a[k].cpu().numpy(), err_msg="replica 2 %s" % k)
    for r in (0, 1):
        for k, v in packed[r].state_dict().items():
            np.testing.assert_array_equal(v.cpu().numpy(), frozen[r][k], err_msg="stopped replica %d %s" % (r, k))
    v = solo.validate_training(val, 1, CFG["p"], *[[] for _ in range(5)])
    np.testing.assert_allclose(losses[2], [v[0], v[1], v[2], v[3], v[4], v[5], v[9]], rtol=1e-6, atol=1e-9)


def test_pack_mixes_phases_and_rejects_mixed_shapes():
    """Replicas in different phases of their schedules run as one launch chain per phase group,
    each bit-identical to its own batch_update sequence; differing shapes are refused."""
    from redcliff_amd import ReplicaPack
    train = data(64 + 24, seed=1)
    solo = [make(0, 10.0, 0.1), make(1, 10.0, 0.1, pre=2)]
    packed = [make(0, 10.0, 0.1), make(1, 10.0, 0.1, pre=2)]
    pack = ReplicaPack(packed, [opts(m, 5e-4, 5e-4) for m in packed])
    ds = pack.cache_dataset(train)
    solo_opts = [opts(m, 5e-4, 5e-4) for m in solo]
    for epoch in range(4):
        groups = pack.run_epoch(epoch, ds)
        if epoch == 1:  # replica 0 acclimates its factors, replica 1 still pretrains the embedder
            assert groups == {("acclimate",): [0], ("pretrain_embedder",): [1]}
        for m, (oA, oB) in zip(solo, solo_opts):
            for bi, (Xb, Yb) in enumerate(train):
                m.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
    torch.cuda.synchronize()
    for r, (m, mp) in enumerate(zip(solo, packed)):
        a, b = m.state_dict(), mp.state_dict()
        for k in a:
            np.testing.assert_array_equal(b[k].cpu().numpy(), a[k].cpu().numpy(), err_msg="replica %d %s" % (r, k))
    c = make(2, 10.0, 0.1)
    c2 = redcliff_amd_model_with_hidden(50)
    with pytest.raises(ValueError, match="share every shape"):
        ReplicaPack([c, c2], [opts(c, 5e-4, 5e-4), opts(c2, 5e-4, 5e-4)])


def redcliff_amd_model_with_hidden(h):
    import redcliff_amd
    K, p = CFG["K"], CFG["p"]
    coeff = {"FORECAST_COEFF": 10.0, "FACTOR_SCORE_COEFF": 100.0, "FACTOR_COS_SIM_COEFF": 1.0 / sum(range(1, K)),
             "FACTOR_WEIGHT_L1_COEFF": 1e-3, "FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF": 0.0,
             "ADJ_L1_REG_COEFF": 0.1 / K / np.sqrt(p * p - 1.0), "DAGNESS_REG_COEFF": 0.0, "DAGNESS_LAG_COEFF": 0.0,
             "DAGNESS_NODE_COEFF": 0.0}
    eargs = [("num_features_per_node", CFG["F"]), ("num_graph_conv_layers", CFG["n"]),
             ("num_hidden_nodes", CFG["H"]), ("sigmoid_eccentricity_coeff", 10.0)]
    torch.manual_seed(5)
    return redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing(
        p, CFG["L"], [h], CFG["F"], [0], CFG["L"], 1, K, CFG["nsup"], coeff, False, "DGCNN", eargs,
        "conditional_factor_fixed_embedder", "apply_factor_weights_after_sim_completion", num_sims=1,
        training_mode="pretrain_embedder_then_acclimate_factors_then_combined", num_pretrain_epochs=1,
        num_acclimation_epochs=1).cuda()


@pytest.mark.parametrize("variant", ["0", "1"])
def test_window_block_combine_variants_bitwise(variant, monkeypatch):
    """The embedder-backward window-block partials can be summed by the last-arriving workgroup
    (REDCLIFF_DEFER=0), a separate k_emb_combine launch (1, the default) or read in
    place by k_emb_final (2): same sums in the same order, so the fits agree bit for bit (ragged
    last batch included)."""
    monkeypatch.setenv("REDCLIFF_FAC_PATH", "vector")
    train = data(64 * 2 + 24, seed=5)
    fits = {}
    for v in ("2", variant):
        monkeypatch.setenv("REDCLIFF_DEFER", v)
        m = make(0, 10.0, 0.1)
        oA, oB = opts(m, 5e-4, 2e-4)
        for epoch in (0, 1, 2, 3):
            for bi, (Xb, Yb) in enumerate(train):
                m.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
        torch.cuda.synchronize()
        fits[v] = {k: t.detach().cpu().numpy() for k, t in m.state_dict().items()}
    for k, want in fits[variant].items():
        np.testing.assert_array_equal(fits["2"][k], want, err_msg=k)


@pytest.mark.parametrize("path", ["vector", "mfma"])
def test_grouped_validation_bitwise_equals_batch_loop(path, monkeypatch):
    """validate_training with the validation batches on the replica axis (runs of <= 7 equal
    batches per launch chain, parameter strides 0; FitEngine._run_values_grouped) against one
    launch chain per batch: identical accumulators and confusion counts, bit for bit, with a
    ragged last batch, after training has moved the parameters off their initial values."""
    monkeypatch.setenv("REDCLIFF_FAC_PATH", path)
    m = make(3, 10.0, 0.1)
    oA, oB = opts(m, 5e-4, 2e-4)
    train = data(64 * 2, seed=11)
    for epoch in (0, 1, 2):
        for bi, (Xb, Yb) in enumerate(train):
            m.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
    val = data(64 * 9 + 40, seed=12)  # 9 full batches (groups of 7 + 2) and a ragged one
    eng = m.engine()
    ds = eng.cache_dataset(val)
    d = eng.workspace(ds["Bmax"], ds["T"])
    acc_g, conf_g = eng.run_values(ds["X"], ds["lab"], d, ds["rows"], ds["sizes"])
    acc_s, conf_s = eng.run_values(ds["X"], ds["lab"], d, ds["rows"], ds["sizes"], grouped=False)
    assert acc_s[7] == len(val)
    np.testing.assert_array_equal(acc_g, acc_s)
    np.testing.assert_array_equal(conf_g, conf_s)
    v1 = m.validate_training(val, 1, m.num_series, [], [], [], [], [])
    assert v1[9] == acc_s[6] / len(val)
