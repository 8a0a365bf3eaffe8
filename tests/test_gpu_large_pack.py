"""The packed-grid code paths the bench's grid and fits/hour legs run (R = 128 D4IC fits per launch),
each held to independent fits or to the path it replaces, bit for bit:

* a real pack of 128 replicas (`k_emb_final` at 8 parameter elements per thread from 96 replicas,
  its batched EF_EPT_MAX gradient loads, rc_embed.hip `rc_launch_emb_final`; the factor chain on the
  second stream from 32 replicas, rc_capi.hip; the GEMM-shaped embedder from 16) through all three
  phases, three sampled replicas against independent single fits on the same factor / embedder path;
* `REDCLIFF_EMB_FINAL_EPT=8` forced on an 8-replica pack against the default (4 elements per thread);
* the forked packed step (factor chain on the second stream) against the single-stream step at R = 32;
* the 256-replica TST-grid pack with mixed phase schedules (the bench's reference-grid pack size)
  against sampled independent fits.
"""
import numpy as np
import pytest
import torch

from test_gpu_replicas import CFG, data, make, opts

pytestmark = pytest.mark.gpu


def grid(R):
    """R grid points (seed, FORECAST_COEFF, ADJ_L1 scale, gen_lr, embed_lr) cycling the reference's
    TST grid values (train/REDCLIFF_S_CMLP_tst100hzRerun1024AvgReg_gsSmooth1.py:283-300)."""
    return [(100 + r, (10.0, 1.0)[r % 2], (0.1, 0.01)[(r // 2) % 2], (5e-4, 1e-4)[(r // 4) % 2],
             (5e-4, 1e-4)[(r // 8) % 2]) for r in range(R)]


def states(models):
    return [{k: t.detach().cpu().numpy() for k, t in m.state_dict().items()} for m in models]


def run_pack(points, train, epochs=(0, 1, 2, 3)):
    from redcliff_amd import ReplicaPack
    models = [make(s, fc, adj) for s, fc, adj, _, _ in points]
    pack = ReplicaPack(models, [opts(m, lrB, lrA) for m, (_, _, _, lrB, lrA) in zip(models, points)])
    ds = pack.cache_dataset(train)
    for epoch in epochs:  # pretrain-embedder, acclimate, combined, combined
        pack.run_epoch(epoch, ds)
    torch.cuda.synchronize()
    return pack, models


def assert_same(a, b, tag):
    assert set(a) == set(b), tag
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg="%s %s" % (tag, k))


def test_pack_of_128_matches_sampled_independent_fits(monkeypatch):
    monkeypatch.setenv("REDCLIFF_FAC_PATH", "mfma")
    monkeypatch.setenv("REDCLIFF_EMB_PATH", "gemm")
    for k in ("REDCLIFF_FORK", "REDCLIFF_EMB_FINAL_EPT"):
        monkeypatch.delenv(k, raising=False)
    points = grid(128)
    train = data(64 * 2 + 24, seed=21)  # two full batches and a ragged one
    val = data(80, seed=22)
    pack, packed = run_pack(points, train)
    vds = pack.cache_dataset(val)
    losses, _ = pack.validate(vds)
    got = states(packed)
    for r in (0, 77, 127):
        s, fc, adj, lrB, lrA = points[r]
        m = make(s, fc, adj)
        oA, oB = opts(m, lrB, lrA)
        for epoch in (0, 1, 2, 3):
            for bi, (Xb, Yb) in enumerate(train):
                m.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
        torch.cuda.synchronize()
        assert_same(got[r], states([m])[0], "replica %d" % r)
        v = m.validate_training(val, 1, CFG["p"], *[[] for _ in range(5)])
        np.testing.assert_allclose(losses[r], [v[0], v[1], v[2], v[3], v[4], v[5], v[9]], rtol=1e-6, atol=1e-9,
                                   err_msg="replica %d losses" % r)
    # replicas that differ in their hyper-parameters really diverged (the pack did not alias rows)
    assert not np.array_equal(got[0]["factors.0.networks.0.layers.0.weight"],
                              got[1]["factors.0.networks.0.layers.0.weight"])


def test_emb_final_eight_elements_per_thread_bitwise(monkeypatch):
    monkeypatch.setenv("REDCLIFF_FAC_PATH", "mfma")
    monkeypatch.setenv("REDCLIFF_EMB_PATH", "gemm")
    points = grid(8)
    train = data(64 * 2 + 24, seed=23)
    out = {}
    for ept in ("8", None):
        if ept is None:
            monkeypatch.delenv("REDCLIFF_EMB_FINAL_EPT", raising=False)
        else:
            monkeypatch.setenv("REDCLIFF_EMB_FINAL_EPT", ept)
        out[ept] = states(run_pack(points, train)[1])
    for r, (a, b) in enumerate(zip(out["8"], out[None])):
        assert_same(a, b, "replica %d" % r)


def test_forked_pack_step_bitwise_equals_single_stream(monkeypatch):
    monkeypatch.setenv("REDCLIFF_FAC_PATH", "mfma")
    monkeypatch.setenv("REDCLIFF_EMB_PATH", "gemm")
    points = grid(32)
    train = data(64 * 2 + 24, seed=24)
    out = {}
    for fork in ("1", "0"):
        monkeypatch.setenv("REDCLIFF_FORK", fork)
        out[fork] = states(run_pack(points, train)[1])
    for r, (a, b) in enumerate(zip(out["1"], out["0"])):
        assert_same(a, b, "replica %d" % r)


def test_tst_pack_of_256_mixed_schedules_matches_sampled_independent_fits(monkeypatch):
    """The pack the bench's reference-grid leg times: 256 points of one TST-grid shape class
    (train/REDCLIFF_S_CMLP_tst100hzRerun1024AvgReg_gsSmooth1.py:278-309: p = 12 region averages, K = 9
    factors of which 3 supervised, h = 25, gen_lag 4, DGCNN embed_lag 16 / 2 graph-conv layers / 100
    hidden), each point with its own learning rates, FORECAST / ADJ_L1 coefficients and its own phase
    schedule (the grid's pretrain x acclimation axes, scaled down: four schedules mixed in one pack,
    Adam step numbers per replica through t_offset) -- ReplicaPack.fit over whole fits with per-epoch
    GC tracking and validation; three sampled replicas (first, middle, last) bit-identical to their
    own independent fit(): histories, stopping epoch, parameters, buffers, Adam moments and steps."""
    import bench
    import redcliff_amd
    from redcliff_amd import ReplicaPack
    from test_gpu_pack_fit import HKEYS, same
    monkeypatch.setenv("REDCLIFF_FAC_PATH", "mfma")
    monkeypatch.setenv("REDCLIFF_EMB_PATH", "gemm")
    for k in ("REDCLIFF_FORK", "REDCLIFF_EMB_FINAL_EPT"):
        monkeypatch.delenv(k, raising=False)
    c = dict(bench.CONFIGS["c4"], F=16, n=2, T=20)
    pts = [q for q in bench.tst_grid_points() if (q["lag"], q["layers"]) == (16, 2)]
    assert len(pts) == 256
    sched = {(100, 15): (2, 1), (100, 100): (2, 2), (50, 15): (1, 1), (50, 100): (1, 2)}
    B = 128
    X, Y = bench.synth(c, 3 * B, seed=401)
    train = [(X[i:i + B], Y[i:i + B]) for i in range(0, 2 * B, B)]
    val = [(X[2 * B:], Y[2 * B:])]
    rng = np.random.RandomState(8)
    gc = [(rng.rand(c["p"], c["p"], c["L"]) < 0.2).astype(np.float64) for _ in range(c["nsup"])]
    kw = dict(lookback=10 ** 6, check_every=10 ** 6, GC=gc, deltaConEps=0.1, verbose=0)
    max_iter = 5

    def model(i):
        q = pts[i]
        pre, acc = sched[(q["pre"], q["acc"])]
        m = bench.build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=7000 + i, pre=pre, acc=acc,
                              forecast=q["forecast"], adj=q["adj"]).cuda()
        return m, bench.adam_pair(m, dict(c, lrA=q["embed_lr"], lrB=q["gen_lr"]))

    made = [model(i) for i in range(256)]
    packed = [m for m, _ in made]
    pack_opts = [o for _, o in made]
    pack = ReplicaPack(packed, pack_opts)
    assert len(pack.phase_groups(1)) > 1  # the schedules really are mixed
    pack.fit(None, train, val, max_iter, **kw)
    torch.cuda.synchronize()
    for r in (0, 131, 255):
        m, (oA, oB) = model(r)
        m.fit(None, train, oA, oB, c["L"], 1, 1, max_iter, val, **kw)
        torch.cuda.synchronize()
        ha, hb = m.fit_history, packed[r].fit_history
        assert hb["best_it"] == ha["best_it"] and hb["stopped_at"] == ha["stopped_at"], r
        for k in HKEYS + ("f1score_histories", "roc_auc_histories", "deltacon0_histories"):
            assert same(hb[k], ha[k]), "replica %d %s" % (r, k)
        assert_same(states([packed[r]])[0], states([m])[0], "replica %d" % r)
        for oa, ob in zip((oA, oB), pack_opts[r]):
            stA, stB = oa.state_dict()["state"], ob.state_dict()["state"]
            for i in stA:
                for k in ("exp_avg", "exp_avg_sq", "step"):
                    np.testing.assert_array_equal(stB[i][k].cpu().numpy(), stA[i][k].cpu().numpy(),
                                                  err_msg="replica %d optimizer state %s %s" % (r, i, k))
