"""fit() in the training modes off the published schedule (models/redcliff_s_cmlp_withStateSmoothing.py
:58-69): the factor re-ordering at the end of factor pretraining ("pretrain_factor" modes,
:1318-1326 -> initialize_factors_with_prior :149-206) and the four Freeze* modes (:910-929,
:1486-1532 -> determine_which_factors_need_updates :1132-1172).

Parity of the re-ordering: the permutation is recomputed here independently (eval-mode
weightings of the first <= 10 training batches against the label columns, the reference's
cosine cost minimised by scipy's linear_sum_assignment, general_utils/metrics.py:274-301) and
the permuted state (parameters and optimizerB moments) is checked slot by slot; a packed fit in
that mode must equal independent fits bit for bit.  The Freeze* modes fail in the reference at
their first decision (np.linalg.norm(ord=1) of the (p, p, 1) lag-free estimates raises
ValueError); the fused fit must raise the same error with the model in the state the
reference's is in at that point."""
import numpy as np
import pytest
import torch
from scipy.optimize import linear_sum_assignment

from test_gpu_pack_fit import HKEYS, same, true_graphs
from test_gpu_replicas import CFG, GRID, data, make, opts

pytestmark = pytest.mark.gpu

REORDER_MODE = "pretrain_factor_then_combined"
PRE = 2


def mk(seed, fc, adj, mode, pre=PRE, acc=0):
    return make(seed, fc, adj, pre=pre, acc=acc, mode=mode)


def expected_order(model, X_train, max_batches=10):
    """initialize_factors_with_prior's matching, restated (misc.py:83-91 with start 0)."""
    Lm = model.Lmax
    preds, labs = [], []
    with torch.no_grad():
        for b, (X, Y) in enumerate(X_train):
            if b >= max_batches:
                break
            if Y.dim() > 2:
                Y = Y[:, :, Lm] if Y.size(2) > Lm else Y[:, :, 0]
            model.factor_score_embedder.eval()
            for f in model.factors:
                f.eval()
            _, _, fw, _ = model.forward(X[:, :Lm, :].cuda().float())
            preds.append(fw[0].cpu().numpy())
            labs.append(Y.cpu().numpy())
    P, Yl = np.vstack(preds), np.vstack(labs)
    cost = np.zeros((P.shape[1], Yl.shape[1]))
    for i in range(P.shape[1]):
        for j in range(Yl.shape[1]):
            a, b = P[:, i], Yl[:, j]  # general_utils/metrics.py:321-339 on the float32 columns
            cost[i, j] = np.dot(a, b) / (max(np.linalg.norm(a), 1e-8) * max(np.linalg.norm(b), 1e-8))
    ei, gi = linear_sum_assignment(cost)
    order = [None] * len(ei)
    for e, g in zip(ei, gi):
        order[g] = int(e)
    return order + [i for i in range(P.shape[1]) if i not in ei]


def factor_state(model, oB):
    """Per factor: its parameters and optimizerB moments, as host arrays."""
    out = []
    for f in model.factors:
        row = []
        for prm in f.parameters():
            st = oB.state.get(prm, {})
            row.append([prm.detach().cpu().numpy().copy()] +
                       [st[k].detach().cpu().numpy().copy() for k in ("exp_avg", "exp_avg_sq") if k in st])
        out.append(row)
    return out


@pytest.mark.parametrize("path", ["vector", "mfma"])
def test_pretrain_factor_reorder(path, monkeypatch):
    import redcliff_amd
    monkeypatch.setenv("REDCLIFF_FAC_PATH", path)
    train, val = data(64 * 3, seed=5), data(64, seed=6)
    cls = redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing
    orig = cls._permute_factors
    seen = []

    def spy(self, order):
        want = expected_order(self, train)
        before = factor_state(self, self._spy_oB)
        orig(self, order)
        after = factor_state(self, self._spy_oB)
        for i, src in enumerate(order):
            for a, b in zip(after[i], before[src]):
                for x, y in zip(a, b):
                    np.testing.assert_array_equal(x, y)
        seen.append((list(order), want))

    monkeypatch.setattr(cls, "_permute_factors", spy)
    for s, fc, adj, lrB, lrA in GRID:
        m = mk(s, fc, adj, REORDER_MODE)
        oA, oB = opts(m, lrB, lrA)
        m._spy_oB = oB
        m.fit(None, train, oA, oB, 4, 1, 1, PRE + 2, val, lookback=1, check_every=1, verbose=0)
        torch.cuda.synchronize()
    assert len(seen) == len(GRID)
    for got, want in seen:
        assert got == want
    print("orders:", [g for g, _ in seen])
    assert any(g != list(range(CFG["K"])) for g, _ in seen), "every matching was the identity"


def test_pretrain_factor_pack_equals_independent_fits(monkeypatch):
    from redcliff_amd import ReplicaPack
    monkeypatch.setenv("REDCLIFF_FAC_PATH", "mfma")
    train, val = data(64 * 2 + 24, seed=3), data(96, seed=4)
    kw = dict(lookback=1, check_every=1, GC=true_graphs(4, 10, 4), deltaConEps=0.1)
    max_iter = PRE + 4
    solo = []
    for s, fc, adj, lrB, lrA in GRID:
        m = mk(s, fc, adj, REORDER_MODE)
        oA, oB = opts(m, lrB, lrA)
        m.fit(None, train, oA, oB, 4, 1, 1, max_iter, val, verbose=0, **kw)
        torch.cuda.synchronize()
        solo.append(m)
    packed = [mk(s, fc, adj, REORDER_MODE) for s, fc, adj, _, _ in GRID]
    pack = ReplicaPack(packed, [opts(m, lrB, lrA) for m, (_, _, _, lrB, lrA) in zip(packed, GRID)])
    pack.fit(None, train, val, max_iter, verbose=0, **kw)
    torch.cuda.synchronize()
    for r, (a, b) in enumerate(zip(solo, packed)):
        ha, hb = a.fit_history, b.fit_history
        assert hb["best_it"] == ha["best_it"] and hb["stopped_at"] == ha["stopped_at"], r
        for k in HKEYS + ("f1score_histories", "roc_auc_histories"):
            assert same(hb[k], ha[k]), "replica %d %s" % (r, k)
        sa, sb = a.state_dict(), b.state_dict()
        for k in sa:
            np.testing.assert_array_equal(sb[k].cpu().numpy(), sa[k].cpu().numpy(), err_msg="replica %d %s" % (r, k))


FREEZE = ["pretrain_embedder_then_post_train_factor_withComboCosSimL1FreezeByEpoch",
          "pretrain_embedder_then_post_train_factor_withComboCosSimL1FreezeByBatch",
          "pretrain_embedder_then_post_train_factor_withL1FreezeByEpoch",
          "pretrain_embedder_then_post_train_factor_withL1FreezeByBatch"]


@pytest.mark.parametrize("mode", FREEZE)
def test_freeze_modes_fail_like_the_reference(mode):
    train, val = data(64 * 2, seed=7), data(64, seed=8)
    s, fc, adj, lrB, lrA = GRID[0]
    m = mk(s, fc, adj, mode, pre=1)
    oA, oB = opts(m, lrB, lrA)
    with pytest.raises(ValueError, match="Improper number of dimensions to norm"):
        m.fit(None, train, oA, oB, 4, 1, 1, 4, val, lookback=1, check_every=1, verbose=0)
    torch.cuda.synchronize()
    # the state the reference's model is left in when the error propagates
    ref = mk(s, fc, adj, "pretrain_embedder_then_post_train_factor", pre=1)
    rA, rB = opts(ref, lrB, lrA)
    if "ByBatch" in mode:  # one embedder-pretraining update (batch 0 of epoch 0), then the decision
        X0, Y0 = train[0]
        ref.batch_update(0, 0, X0, Y0, rA, rB, 1)
    else:  # the pretraining epoch and the first post-training epoch, then the decision
        ref.fit(None, train, rA, rB, 4, 1, 1, 2, val, lookback=1, check_every=1, verbose=0)
    torch.cuda.synchronize()
    sa, sb = m.state_dict(), ref.state_dict()
    for k in sa:
        np.testing.assert_array_equal(sa[k].cpu().numpy(), sb[k].cpu().numpy(), err_msg=k)


@pytest.mark.parametrize("name", ["cemb", "vanilla"])
def test_reorder_on_the_generic_path(name):
    """Configurations outside the fused chain re-order the factor modules themselves, as the
    reference does (:200-205): module i of the new list is old module order[i]."""
    from golden_io import batches, load
    from test_gpu_generic import build
    d, meta = load(name)
    m = build(meta)
    bs = batches(d, meta)
    want = expected_order(m, bs)
    old = list(m.factors)
    m.initialize_factors_with_prior(X_train=bs)
    assert [id(f) for f in m.factors] == [id(old[i]) for i in want]


@pytest.mark.parametrize("form", ["state_dict", "module"])
def test_prior_factors_path(form, tmp_path, monkeypatch):
    """fit(prior_factors_path=...) (:1318-1326 at epoch 0 -> :149-206).  The reference replaces
    the factors by the saved model's and re-orders them; its optimizerB still holds the replaced
    parameters, so the loaded factors never change again, while the embedder keeps training
    against them.  Twin: the same model given the permuted prior factors by hand and trained
    with optimizerB at lr 0 (the fused Adam then leaves the factors bit-identical), so the
    embedder's updates through the optimizerB-less steps must match it bit for bit.
    form "state_dict": the prior's state_dict, loaded weights-only (the default); "module": the
    pickled module the reference writes, loaded only with prior_factors_allow_pickle=True."""
    monkeypatch.setenv("REDCLIFF_FAC_PATH", "mfma")
    train, val = data(64 * 2, seed=12), data(64, seed=13)
    s, fc, adj, lrB, lrA = GRID[0]
    mode = "pretrain_embedder_then_acclimate_factors_then_combined"
    prior = mk(9, fc, adj, mode, pre=1, acc=1)
    path = str(tmp_path / "prior.bin")
    torch.save(prior.state_dict() if form == "state_dict" else prior, path)
    pf = [[p.detach().cpu().numpy().copy() for p in f.parameters()] for f in prior.factors]

    m = mk(s, fc, adj, mode, pre=1, acc=1)
    order = expected_order(m, train)
    oA, oB = opts(m, lrB, lrA)
    if form == "module":  # a pickled module needs the explicit opt-in
        m0 = mk(s, fc, adj, mode, pre=1, acc=1)
        a0, b0 = opts(m0, lrB, lrA)
        with pytest.raises(RuntimeError, match="prior_factors_allow_pickle"):
            m0.fit(None, train, a0, b0, 4, 1, 1, 4, val, lookback=1, check_every=1, verbose=0, prior_factors_path=path)
    m.fit(None, train, oA, oB, 4, 1, 1, 4, val, lookback=1, check_every=1, verbose=0, prior_factors_path=path,
          prior_factors_allow_pickle=(form == "module"))
    torch.cuda.synchronize()
    for i, f in enumerate(m.factors):
        for got, want in zip(f.parameters(), pf[order[i]]):
            np.testing.assert_array_equal(got.detach().cpu().numpy(), want)

    twin = mk(s, fc, adj, mode, pre=1, acc=1)
    with torch.no_grad():
        for i, f in enumerate(twin.factors):
            for p, want in zip(f.parameters(), pf[order[i]]):
                p.copy_(torch.from_numpy(want))
    tA, tB = opts(twin, 0.0, lrA)
    twin.fit(None, train, tA, tB, 4, 1, 1, 4, val, lookback=1, check_every=1, verbose=0)
    torch.cuda.synchronize()
    sa, sb = m.state_dict(), twin.state_dict()
    for k in sa:
        np.testing.assert_array_equal(sa[k].cpu().numpy(), sb[k].cpu().numpy(), err_msg=k)
    assert m.fit_history["avg_combo_loss"] == twin.fit_history["avg_combo_loss"]
