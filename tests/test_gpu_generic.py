"""The generic GPU path (redcliff_amd.generic: HIP GEMM contractions, autograd) against the
reference's golden vectors, for every configuration outside the fused chain:
cEmbedder, the Vanilla embedders, num_sims = 2 roll-outs with the smoothing penalty, and the
per-step factor weighting forward mode (models/redcliff_s_cmlp_withStateSmoothing.py:253-412,
models/redcliff_factor_score_embedders.py:51-331).

Tolerance as the fused-path tests: rtol 1e-4 (north star), atol 1e-5 on near-zero entries."""
import numpy as np
import pytest
import torch

from golden_io import assert_close, batches, ctor_args, load, state

pytestmark = pytest.mark.gpu

GENERIC_SCENARIOS = ["cemb", "vanilla", "dgcnn_sims2", "dgcnn_eachstep"]
RTOL, ATOL = 1e-4, 1e-5


def build(meta):
    import redcliff_amd
    args, kw = ctor_args(meta)
    torch.manual_seed(meta["seed"])
    cls = redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing if meta["smoothing_class"] else redcliff_amd.REDCLIFF_S_CMLP
    m = cls(*args, **kw).float().cuda()
    assert not m.fused_supported(), "scenario is expected to run on the generic path"
    return m


def compare_state(tag, model, want, rtol=RTOL, atol=ATOL):
    got = dict((k, v.detach().cpu().numpy()) for k, v in model.state_dict().items() if not k.startswith("gen_model."))
    assert set(got) == set(want)
    for k in want:
        if k.endswith("num_batches_tracked"):
            assert int(got[k]) == int(want[k]), tag + k
            continue
        scale = max(1.0, float(np.abs(want[k]).max()))
        assert_close("%s/%s" % (tag, k), got[k], want[k], rtol, atol * scale)


@pytest.mark.parametrize("name", GENERIC_SCENARIOS)
def test_init_is_the_reference_init(name):
    d, meta = load(name)
    compare_state("init", build(meta), state(d, "init"), rtol=0, atol=0)


@pytest.mark.parametrize("name", GENERIC_SCENARIOS)
def test_eval_forward_gc_loss(name):
    d, meta = load(name)
    m = build(meta)
    m.eval()
    Xb, Yb = batches(d, meta)[0]
    Lm = max(meta["L"], meta["F"])
    X = Xb[:, :Lm, :].cuda()
    with torch.no_grad():
        x_sim, fpreds, fws, labels = m(X)
        assert_close("x_sim", x_sim.cpu().numpy(), d["eval/x_sim"], RTOL, ATOL)
        assert_close("w", fws[0].cpu().numpy(), d["eval/w"], RTOL, ATOL)
        assert_close("labels0", labels[0].cpu().numpy(), d["eval/labels0"], RTOL, ATOL)
        for key in [k for k in d.files if k.startswith("eval/gc/")]:
            _, _, mode, ign, comb = key.split("/")
            gcs = m.GC(mode, X=X, threshold=False, ignore_lag=ign == "ign1",
                       combine_wavelet_representations=comb == "comb1")
            arr = np.stack([np.stack([g.detach().cpu().numpy() for g in row]) for row in gcs])
            assert_close(key, arr, d[key], RTOL, ATOL)
        tgt = Xb[:, Lm:Lm + meta["S"], :].cuda()
        for flag in ("combined", "emb", "fac"):
            combo, terms = m.compute_loss(X[:, :meta["F"], :], x_sim, tgt, labels, Yb.cuda(), meta["gc_mode"],
                                          embedder_pretrain_loss=flag == "emb", factor_pretrain_loss=flag == "fac")
            assert_close("combo/" + flag, float(combo), d["eval/loss/%s/combo" % flag], RTOL, ATOL)
            for i, t in enumerate(terms):
                want = d["eval/loss/%s/t%d" % (flag, i)]
                if np.isnan(want):
                    assert t is None
                else:
                    assert_close("term%d/%s" % (i, flag), float(t), want, RTOL, ATOL)


@pytest.mark.parametrize("name", GENERIC_SCENARIOS)
def test_train_mode_forward(name):
    d, meta = load(name)
    m = build(meta)
    m.train()
    Xb, _ = batches(d, meta)[0]
    with torch.no_grad():
        x_sim, _, fws, _ = m(Xb[:, :max(meta["L"], meta["F"]), :].cuda())
    assert_close("train x_sim", x_sim.cpu().numpy(), d["train_fwd/x_sim"], RTOL, ATOL)
    assert_close("train w", fws[0].cpu().numpy(), d["train_fwd/w"], RTOL, ATOL)


@pytest.mark.parametrize("name", GENERIC_SCENARIOS)
def test_batch_update_schedule_and_validation(name):
    d, meta = load(name)
    m = build(meta)
    oA = torch.optim.Adam(m.gen_model[0].parameters(), lr=meta["lrA"], betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    oB = torch.optim.Adam(m.gen_model[1].parameters(), lr=meta["lrB"], betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    bs = batches(d, meta)
    step = 0
    for epoch in meta["epochs"]:
        for bi, (Xb, Yb) in enumerate(bs):
            m.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
            step += 1
            compare_state("step%d" % step, m, state(d, "step%d" % step))
    assert step == int(d["nsteps"])
    hist = [[] for _ in range(5)] if meta["nsup"] > 0 else []
    vals = m.validate_training(bs, 1, meta["p"], *hist)
    names = ["forecast", "factor", "cos", "fw_l1", "smooth", "adj", "dag_reg", "dag_lag", "dag_node", "combo"]
    if not meta["smoothing_class"]:
        names = ["forecast", "factor", "cos", "fw_l1", "adj", "dag_reg", "dag_lag", "dag_node", "combo"]
    for n_, v in zip(names, vals):
        if ("val/" + n_) in d.files:
            assert_close("val/" + n_, v, d["val/" + n_], 1e-4, 1e-6)


def test_hip_gemm_against_fp64():
    """redcliff_gemm in all four transpose combinations, batched and broadcast."""
    from redcliff_amd.generic import _raw_bmm, bmm
    g = torch.Generator().manual_seed(0)
    for (M, N, K) in ((1, 1, 1), (7, 65, 33), (64, 64, 16), (130, 3, 257)):
        for ta in (0, 1):
            for tb in (0, 1):
                a = torch.randn((3,) + ((K, M) if ta else (M, K)), generator=g)
                b = torch.randn((1,) + ((N, K) if tb else (K, N)), generator=g)
                got = _raw_bmm(a.cuda(), b.cuda(), ta, tb).cpu().double()
                A = a.double().transpose(1, 2) if ta else a.double()
                Bm = b.double().transpose(1, 2) if tb else b.double()
                # fp32 fmaf chain over K terms vs fp64: |err| <~ K * 2^-24 * sum|a b|
                np.testing.assert_allclose(got.numpy(), torch.matmul(A, Bm).numpy(), rtol=1e-4, atol=1e-4)
    a = torch.randn(1, 9, 5, generator=g).cuda().requires_grad_()
    b = torch.randn(4, 5, 6, generator=g).cuda().requires_grad_()
    (bmm(a, b) ** 2).sum().backward()
    a2, b2 = a.detach().cpu().double().requires_grad_(), b.detach().cpu().double().requires_grad_()
    (torch.matmul(a2, b2) ** 2).sum().backward()
    np.testing.assert_allclose(a.grad.cpu().numpy(), a2.grad.numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(b.grad.cpu().numpy(), b2.grad.numpy(), rtol=1e-5, atol=1e-5)


def test_gemm_cores_bitwise(monkeypatch):
    """The matrix-core GEMM (k_rc_gemm_mfma: 32x32x2 / 16x16x4 fp32 MFMA), the vector-ALU
    one (k_rc_gemm, REDCLIFF_GEMM_CORE=valu) and the wave core (k_rc_gemm_wave, one wave per
    32x32 tile, k-contiguous operands transposed through the wave's LDS tile: REDCLIFF_GEMM_CORE=wave;
    every operand loaded straight into the lanes: wd) give the same bits: all are in-order fmaf chains
    over k.  Shapes cover both tile sizes (64x64 tiles when the launch has >= 512 of them),
    ragged edges and all transpose combinations."""
    from redcliff_amd.generic import _raw_bmm
    g = torch.Generator().manual_seed(1)
    shapes = ((1, 1, 1, 3), (7, 65, 33, 3), (64, 64, 16, 3), (130, 3, 257, 3), (200, 300, 70, 2),
              (256, 256, 40, 32), (100, 260, 129, 40))
    for (M, N, K, nb) in shapes:
        for ta in (0, 1):
            for tb in (0, 1):
                a = torch.randn((nb,) + ((K, M) if ta else (M, K)), generator=g).cuda()
                b = torch.randn((nb,) + ((N, K) if tb else (K, N)), generator=g).cuda()
                monkeypatch.delenv("REDCLIFF_GEMM_CORE", raising=False)
                got = _raw_bmm(a, b, ta, tb).cpu().numpy()
                for core in ("valu", "wave", "wd", "mfma"):
                    monkeypatch.setenv("REDCLIFF_GEMM_CORE", core)
                    want = _raw_bmm(a, b, ta, tb).cpu().numpy()
                    np.testing.assert_array_equal(got, want, err_msg="%s M=%d N=%d K=%d ta=%d tb=%d" % (core, M, N, K, ta, tb))


@pytest.mark.parametrize("name", ["cemb", "vanilla"])
def test_hip_adam_matches_torch_adam(name, monkeypatch):
    """The generic path's optimizer steps (generic.HipAdam: flat parameter / moment buffers, one
    redcliff_adam_apply launch per group) against torch.optim.Adam's own step on a twin model: the
    same schedule of batch_updates, parameters and Adam moments within 2 ulp-scale tolerances (the
    per-element formula is torch's single-tensor Adam; torch's CUDA Adam is the multi-tensor form),
    the step counts equal, and the optimizers' state_dict() keeps its structure."""
    from redcliff_amd import generic
    d, meta = load(name)
    runs = []
    for hip in (True, False):
        m = build(meta)
        oA = torch.optim.Adam(m.gen_model[0].parameters(), lr=meta["lrA"], betas=(0.9, 0.999), eps=1e-4,
                              weight_decay=1e-4)
        oB = torch.optim.Adam(m.gen_model[1].parameters(), lr=meta["lrB"], betas=(0.9, 0.999), eps=1e-4,
                              weight_decay=1e-4)
        if not hip:
            monkeypatch.setattr(generic.GenericPath, "_step", lambda self, opt: opt.step())
        for epoch in range(meta["pre"] + meta["acc"] + 2):
            for bi, (Xb, Yb) in enumerate(batches(d, meta)):
                m.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
        torch.cuda.synchronize()
        monkeypatch.undo()
        runs.append((m, oA, oB))
    (ma, aA, aB), (mb, bA, bB) = runs
    # HipAdam was in charge of both groups, except one that met a step where some parameter had no
    # gradient (a phase that leaves part of the Vanilla embedder out of the loss; torch skips those
    # parameters, weight decay included): that one went back to torch for good
    g = ma._generic()
    assert len(g._adams) == 2 and all(h is not None for h in g._adams.values())
    assert any(h.ok for h in g._adams.values())
    for h in g._adams.values():
        assert h.ok or h.released_for == "missing gradient", h.released_for
    sa, sb = ma.state_dict(), mb.state_dict()
    for k in sb:
        w = sb[k].detach().cpu().numpy().astype(np.float64)
        scale = max(1.0, float(np.abs(w).max()))
        assert_close("param " + k, sa[k].detach().cpu().numpy(), w, 1e-5, 1e-7 * scale)
    for oa, ob in ((aA, bA), (aB, bB)):
        da, db = oa.state_dict(), ob.state_dict()
        assert da["param_groups"] == db["param_groups"] and da["state"].keys() == db["state"].keys()
        for i in db["state"]:
            assert float(da["state"][i]["step"]) == float(db["state"][i]["step"])
            for k in ("exp_avg", "exp_avg_sq"):
                w = db["state"][i][k].cpu().numpy().astype(np.float64)
                assert_close("%s %s" % (i, k), da["state"][i][k].cpu().numpy(), w, 1e-4,
                             1e-7 * max(1.0, float(np.abs(w).max())))


def test_hip_adam_reloaded_state_and_unequal_steps():
    """generic.HipAdam and torch.optim.Adam's own state handling:
      * optimizer.load_state_dict() on an optimizer HipAdam already steps swaps new moment / step
        tensors into its state; the next step continues from the LOADED moments and step count
        (GenericPath._step rebuilds on them), as torch's Adam does;
      * an optimizer torch stepped with a parameter left out (no gradient: torch skips it) has
        per-parameter step counts that differ, which one flat launch cannot reproduce: it stays
        with torch."""
    from redcliff_amd import generic
    gp = generic.GenericPath(None)
    g = torch.Generator().manual_seed(5)
    init = [torch.randn(7, 5, generator=g), torch.randn(11, generator=g)]
    grads = [[torch.randn(t.shape, generator=g) for t in init] for _ in range(6)]

    def make():
        ps = [torch.nn.Parameter(t.clone().cuda()) for t in init]
        return ps, torch.optim.Adam(ps, lr=1e-2, betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)

    (pa, oa), (pb, ob) = make(), make()
    saved = None
    for i, gr in enumerate(grads):
        if i == 4:  # both optimizers reload the twin's state of step 2
            oa.load_state_dict(saved)
            ob.load_state_dict(saved)
            with torch.no_grad():
                for x, y in zip(pa, pb):
                    x.copy_(y)
        for ps in (pa, pb):
            for p, t in zip(ps, gr):
                p.grad = t.cuda()
        gp._step(oa)
        ob.step()
        if i == 1:
            import copy
            saved = copy.deepcopy(ob.state_dict())
    torch.cuda.synchronize()
    h = gp._adams[id(oa)]
    assert h.ok and h.state_is_ours() and h.t == 4
    for x, y in zip(pa, pb):
        np.testing.assert_allclose(x.detach().cpu().numpy(), y.detach().cpu().numpy(), rtol=1e-6, atol=1e-7)
    for i in ob.state_dict()["state"]:
        sa, sb = oa.state_dict()["state"][i], ob.state_dict()["state"][i]
        assert float(sa["step"]) == float(sb["step"]) == 4.0
        for k in ("exp_avg", "exp_avg_sq"):
            np.testing.assert_allclose(sa[k].cpu().numpy(), sb[k].cpu().numpy(), rtol=1e-6, atol=1e-9)
    # unequal per-parameter step counts stay with torch
    ps, oc = make()
    for i in range(3):
        ps[0].grad = grads[i][0].cuda()
        ps[1].grad = grads[i][1].cuda() if i != 1 else None
        oc.step()
    assert float(oc.state[ps[0]]["step"]) == 3.0 and float(oc.state[ps[1]]["step"]) == 2.0
    h = generic.HipAdam(oc)
    assert not h.ok and h.released_for.startswith("unequal step counts")


@pytest.mark.parametrize("shape", ["c5", "d4ic-products", "d4ic-pack"])
def test_gemm_product_sets_bitwise(shape, monkeypatch):
    """rc_gemm_launch_set: the GEMM-shaped embedder's independent products in one launch (forward: the
    T_i = S_i x_bn products; backward: dfc1W with dZ, dW with dT, dx_bn with the dS_i slices) against
    one launch per product (REDCLIFF_GEMM_SET=0) -- the same body and k order per output, so three
    combined-phase steps end bit-identical.  "c5": configs[4] (p = 64, the single fit's default GEMM
    embedder); "d4ic-products": the D4IC shape with the GEMM products forced (REDCLIFF_EMB_PATH=gemm,
    REDCLIFF_EMB_WIN=0); "d4ic-pack": a 16-replica D4IC pack on the GEMM embedder, whose pairs run on
    the wave core (k_rc_gemm_wave_pair)."""
    import bench
    import redcliff_amd
    c = dict(bench.CONFIGS["c5" if shape == "c5" else "d4ic"])
    if shape != "c5":
        monkeypatch.setenv("REDCLIFF_EMB_PATH", "gemm")
    if shape == "d4ic-products":
        monkeypatch.setenv("REDCLIFF_EMB_WIN", "0")
    X, Y = bench.synth(c, 2 * c["B"], seed=3)
    R = 16 if shape == "d4ic-pack" else 1
    out = []
    for on in ("1", "0"):
        monkeypatch.setenv("REDCLIFF_GEMM_SET", on)
        ms = [bench.build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=s_).cuda() for s_ in range(R)]
        ops = [bench.adam_pair(m, c) for m in ms]
        if R == 1:
            m, (oA, oB) = ms[0], ops[0]
            for ep, bi in ((0, 0), (1, 1), (2, 0)):  # pretrain, acclimate, combined
                m.batch_update(ep, bi, X[bi * c["B"]:(bi + 1) * c["B"]], Y[bi * c["B"]:(bi + 1) * c["B"]], oA, oB, 1)
        else:
            pack = redcliff_amd.ReplicaPack(ms, ops)
            ds = pack.cache_dataset([(X[i:i + c["B"]], Y[i:i + c["B"]]) for i in range(0, X.shape[0], c["B"])])
            for ep in (0, 1, 2):
                pack.run_epoch(ep, ds)
        torch.cuda.synchronize()
        out.append([dict((k, v.detach().cpu().numpy()) for k, v in m.state_dict().items()) for m in ms])
    for r in range(R):
        for k in out[0][r]:
            np.testing.assert_array_equal(out[0][r][k], out[1][r][k], err_msg="replica %d %s" % (r, k))

