"""The packed-grid code paths the bench's grid and fits/hour legs run (R = 128 D4IC fits per launch),
each held to independent fits or to the path it replaces, bit for bit:

* a real pack of 128 replicas (`k_emb_final` at 8 parameter elements per thread from 96 replicas,
  its batched EF_EPT_MAX gradient loads, rc_embed.hip `rc_launch_emb_final`; the factor chain on the
  second stream from 32 replicas, rc_capi.hip; the GEMM-shaped embedder from 16) through all three
  phases, three sampled replicas against independent single fits on the same factor / embedder path;
* `REDCLIFF_EMB_FINAL_EPT=8` forced on an 8-replica pack against the default (4 elements per thread);
* the forked packed step (factor chain on the second stream) against the single-stream step at R = 32.
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
