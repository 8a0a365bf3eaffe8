"""Two-stream (forked) steps against single-stream steps, bit for bit, under workspace guard bands.

Round 1 saw, twice in a dozen runs, a forked matrix-core fit whose DGCNN adjacency A differed
from the same fit run on one stream.  The cause was a missing barrier in k_emb_final's
adjacency workgroup (rc_embed.hip): the relu(A) row sums read LDS entries other waves had not
stored yet.  Concurrent work on the second stream made the late waves likelier, hence the
apparent link with the fork.  These tests pin the fixed behaviour:

* the verification layout (redcliff_debug_guard_bands) puts a NaN-pattern guard band after
  every workspace region of every replica, the last band closing replica R-1's slice; after
  the run every band must be untouched (no write past a region) and every parameter finite
  (no NaN read from a band);
* a forked single fit (matrix-core factor path, REDCLIFF_FORK=1), also with the in-kernel
  ticket combine (REDCLIFF_DEFER=0), equals the single-stream fit bit for bit through the
  pretrain -> acclimate -> combined schedule (ragged last batch included);
* a forked R = 3 pack equals the single-stream R = 3 pack and the independent fits.
"""
import numpy as np
import pytest
import torch

from test_gpu_replicas import data, make, opts

pytestmark = pytest.mark.gpu

BAND = 64
NAN_BITS = 0x7FC0BEEF  # a quiet NaN with a recognisable payload


@pytest.fixture
def guard_bands():
    from redcliff_amd import _native as nat
    prev = nat.guard_bands(BAND)
    yield BAND
    nat.guard_bands(prev)


def arm(ws, dims, R):
    """Fill the guard band after every region of every replica with the NaN pattern."""
    from redcliff_amd import _native as nat
    regs = nat.workspace_regions(dims)
    total = nat.workspace_layout(dims)["total"]
    assert ws.numel() >= R * total
    iv = ws.view(torch.int32)
    for r in range(R):
        for s, n in regs:
            iv[r * total + s + n:r * total + s + n + BAND] = NAN_BITS
    return regs, total


def check_bands(ws, regs, total, R, tag):
    from redcliff_amd import _native as nat
    iv = ws.view(torch.int32).cpu().numpy()
    names = nat.WS_REGIONS
    for r in range(R):
        for i, (s, n) in enumerate(regs):
            band = iv[r * total + s + n:r * total + s + n + BAND]
            bad = int((band != NAN_BITS).sum())
            name = names[i] if i < len(names) - 1 else "region%d" % i
            assert bad == 0, "%s: replica %d wrote %d floats past the end of workspace region %s" % (tag, r, bad, name)


def run_single(monkeypatch, fork, defer, train, guarded):
    monkeypatch.setenv("REDCLIFF_FAC_PATH", "mfma")
    monkeypatch.setenv("REDCLIFF_FORK", fork)
    monkeypatch.setenv("REDCLIFF_DEFER", defer)
    m = make(0, 10.0, 0.1)
    oA, oB = opts(m, 5e-4, 2e-4)
    eng = m.engine()
    eng.workspace(max(x.shape[0] for x, _ in train), train[0][0].shape[1])
    armed = arm(eng.ws, eng.dims(eng.ws_dims[0], train[0][0].shape[1]), 1) if guarded else None
    for epoch in (0, 1, 2, 3, 4):
        for bi, (Xb, Yb) in enumerate(train):
            m.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
    torch.cuda.synchronize()
    if guarded:
        check_bands(eng.ws, armed[0], armed[1], 1, "fork=%s defer=%s" % (fork, defer))
    st = {k: t.detach().cpu().numpy() for k, t in m.state_dict().items()}
    for k, v in st.items():
        if v.dtype.kind == "f":
            assert np.isfinite(v).all(), k
    return st


@pytest.mark.parametrize("defer", ["1", "0"])
def test_forked_single_fit_bitwise_equals_single_stream(defer, monkeypatch, guard_bands):
    train = data(64 * 2 + 24, seed=7)
    one = run_single(monkeypatch, "0", "1", train, True)
    two = run_single(monkeypatch, "1", defer, train, True)
    for k, want in one.items():
        np.testing.assert_array_equal(two[k], want, err_msg=k)


def test_forked_pack_bitwise_equals_single_stream_pack(monkeypatch, guard_bands):
    from redcliff_amd import ReplicaPack
    from test_gpu_replicas import GRID
    monkeypatch.setenv("REDCLIFF_FAC_PATH", "mfma")
    train = data(64 * 2 + 24, seed=3)
    states = {}
    for fork in ("0", "1"):
        monkeypatch.setenv("REDCLIFF_FORK", fork)
        models = [make(s, fc, adj) for s, fc, adj, _, _ in GRID]
        pack = ReplicaPack(models, [opts(m, lrB, lrA) for m, (_, _, _, lrB, lrA) in zip(models, GRID)])
        ds = pack.cache_dataset(train)
        d = pack._workspace(max(int(ds["Bmax"]), 1), ds["T"])
        regs, total = arm(pack.ws, d, pack.R)
        for epoch in (0, 1, 2, 3):
            pack.run_epoch(epoch, ds)
        torch.cuda.synchronize()
        check_bands(pack.ws, regs, total, pack.R, "pack fork=%s" % fork)
        states[fork] = [{k: t.detach().cpu().numpy() for k, t in m.state_dict().items()} for m in models]
    for r in range(len(GRID)):
        for k, want in states["0"][r].items():
            np.testing.assert_array_equal(states["1"][r][k], want, err_msg="replica %d %s" % (r, k))


def run_vector(monkeypatch, merge, train, guarded, seed=0, split="0", tail="0", ext="1"):
    monkeypatch.setenv("REDCLIFF_FAC_PATH", "vector")
    monkeypatch.setenv("REDCLIFF_MERGE", merge)
    monkeypatch.setenv("REDCLIFF_SPLIT_LEAD", split)
    monkeypatch.setenv("REDCLIFF_TAIL", tail)
    monkeypatch.setenv("REDCLIFF_EXT_EVENT", ext)
    m = make(seed, 10.0, 0.1)
    oA, oB = opts(m, 5e-4, 2e-4)
    eng = m.engine()
    eng.workspace(max(x.shape[0] for x, _ in train), train[0][0].shape[1])
    armed = arm(eng.ws, eng.dims(eng.ws_dims[0], train[0][0].shape[1]), 1) if guarded else None
    for epoch in (0, 1, 2, 3, 4):
        for bi, (Xb, Yb) in enumerate(train):
            m.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
    torch.cuda.synchronize()
    if guarded:
        check_bands(eng.ws, armed[0], armed[1], 1, "merge=%s split=%s tail=%s ext=%s" % (merge, split, tail, ext))
    return {k: t.detach().cpu().numpy() for k, t in m.state_dict().items()}


def test_merged_backward_bitwise_equals_two_launches(monkeypatch, guard_bands):
    """k_bwd_merged (factor and embedder backward in one launch, the embedder workgroups waiting
    on the factor-lead workgroups' published records) against the two dependent launches
    (REDCLIFF_MERGE=0): bit for bit through pretrain -> acclimate -> combined, ragged last
    batch included, with every workspace guard band intact; then a second merged run (the
    lead counter re-arms every step, so repeated steps see fresh records)."""
    train = data(64 * 2 + 24, seed=5)
    two = run_vector(monkeypatch, "0", train, True)
    one = run_vector(monkeypatch, "1", train, True)
    again = run_vector(monkeypatch, "1", train, False)
    for k, want in two.items():
        np.testing.assert_array_equal(one[k], want, err_msg=k)
        np.testing.assert_array_equal(again[k], want, err_msg=k)


def test_split_lead_bitwise_equals_one_launch(monkeypatch, guard_bands):
    """Split-lead step (the factor leads' records in their own launch, the factor update on the
    second stream beside the embedder backward, joined before k_emb_final) against the single
    factor-backward launch on one stream: bit for bit through pretrain -> acclimate -> combined,
    ragged last batch included, guard bands intact; a second split run repeats the first."""
    train = data(64 * 2 + 24, seed=9)
    one = run_vector(monkeypatch, "0", train, True, split="0")
    two = run_vector(monkeypatch, "0", train, True, split="1")
    again = run_vector(monkeypatch, "0", train, False, split="1")
    for k, want in one.items():
        np.testing.assert_array_equal(two[k], want, err_msg=k)
        np.testing.assert_array_equal(again[k], want, err_msg=k)


def test_kernel_completed_events_bitwise(monkeypatch, guard_bands):
    """The split-lead step's fork / join events completed by the forward and factor-update kernels
    themselves (hipExtLaunchKernel stop events, the default) against event-record packets on the
    streams (REDCLIFF_EXT_EVENT=0): bit for bit through pretrain -> acclimate -> combined, guard
    bands intact, a second run repeating the first."""
    train = data(64 * 2 + 24, seed=17)
    want = run_vector(monkeypatch, "0", train, True, split="1", ext="0")
    got = run_vector(monkeypatch, "0", train, True, split="1", ext="1")
    again = run_vector(monkeypatch, "0", train, False, split="1", ext="1")
    for k, w in want.items():
        np.testing.assert_array_equal(got[k], w, err_msg=k)
        np.testing.assert_array_equal(again[k], w, err_msg=k)


@pytest.mark.parametrize("merge,split", [("1", "0"), ("0", "0"), ("0", "1")])
def test_embedder_tail_bitwise_equals_combine_and_final(merge, split, monkeypatch, guard_bands):
    """k_emb_tail (the window-block combine and the embedder optimizer in one launch: the
    adjacency workgroup sums its dS partials in place, the parameter workgroups wait for the
    combine workgroups' published records) against k_emb_combine + k_emb_final: bit for bit
    through pretrain -> acclimate -> combined on the merged, two-launch and split-lead backward
    paths, guard bands intact; a second tail run repeats the first (the counter re-arms)."""
    train = data(64 * 2 + 24, seed=13)
    two = run_vector(monkeypatch, merge, train, True, split=split, tail="0")
    one = run_vector(monkeypatch, merge, train, True, split=split, tail="1")
    again = run_vector(monkeypatch, merge, train, False, split=split, tail="1")
    for k, want in two.items():
        np.testing.assert_array_equal(one[k], want, err_msg=k)
        np.testing.assert_array_equal(again[k], want, err_msg=k)
