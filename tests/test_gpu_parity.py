"""GPU parity of the fused gfx950 REDCLIFF-S path against the reference's golden vectors
and against the CPU oracle on the same seeded inputs.

Tolerance (north star): losses / GC tensors within 1e-4 relative in fp32; parameters
after N Adam steps within rtol 1e-4 (atol 2e-6 for near-zero entries, set by fp32
re-association of batch reductions); thresholded graphs / F1 identical.
All compute goes through libredcliff_hip.so (the tests fail if it is not loaded).
"""
import copy
import os
import re

import numpy as np
import pytest
import torch

from golden_io import assert_close, batches, ctor_args, load, state

pytestmark = pytest.mark.gpu

FUSED_SCENARIOS = ["dgcnn_c1", "dgcnn_d4ic", "dgcnn_partial_sigmoid", "dgcnn_unsup", "dgcnn_base", "dgcnn_feql",
                   "dgcnn_k1p3", "dgcnn_k10p6"]
RTOL, ATOL = 1e-4, 2e-6


def build(meta, device="cuda"):
    import redcliff_amd
    args, kw = ctor_args(meta)
    torch.manual_seed(meta["seed"])
    cls = redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing if meta["smoothing_class"] else redcliff_amd.REDCLIFF_S_CMLP
    return cls(*args, **kw).float().to(device)


def make_opts(m, lrA, lrB):
    oA = torch.optim.Adam(m.gen_model[0].parameters(), lr=lrA, betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    oB = torch.optim.Adam(m.gen_model[1].parameters(), lr=lrB, betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    return oA, oB


def compare_state(tag, model, want, rtol=RTOL, atol=ATOL, outliers=0):
    got = dict((k, v.detach().cpu().numpy()) for k, v in model.state_dict().items() if not k.startswith("gen_model."))
    assert set(got) == set(want)
    for k in want:
        if k.endswith("num_batches_tracked"):
            assert int(got[k]) == int(want[k]), tag + k
            continue
        scale = max(1.0, float(np.abs(want[k]).max()))
        assert_close("%s/%s" % (tag, k), got[k], want[k], rtol, atol * scale, outliers)


def test_native_library_is_the_compute_path():
    from redcliff_amd import _native as nat
    L = nat.lib()
    assert L is not None
    import os
    maps = open("/proc/self/maps").read()
    assert os.path.basename(nat.LIB_PATH) in maps


def test_loaded_library_was_built_from_this_tree():
    """The binary this GPU process runs is the one compiled from the committed sources: its
    embedded build id (redcliff_build_id) equals the hash of csrc/ + include/ on this box."""
    from redcliff_amd import _native as nat
    from redcliff_amd import build as b
    assert not os.environ.get("REDCLIFF_HIP_LIB"), "experiment library selected"
    assert nat.build_id() == b.source_hash()
    maps = open("/proc/self/maps").read()
    assert os.path.realpath(b.LIB) in maps


@pytest.mark.parametrize("name", FUSED_SCENARIOS)
def test_batch_update_schedule_matches_reference(name):
    d, meta = load(name)
    m = build(meta)
    oA, oB = make_opts(m, meta["lrA"], meta["lrB"])
    bs = batches(d, meta)
    step = 0
    for epoch in meta["epochs"]:
        for bi, (Xb, Yb) in enumerate(bs):
            m.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
            step += 1
            compare_state("step%d" % step, m, state(d, "step%d" % step))
    hist = [[] for _ in range(5)] if meta["nsup"] > 0 else []
    vals = m.validate_training(bs, 1, meta["p"], *hist)
    names = ["forecast", "factor", "cos", "fw_l1", "smooth", "adj", "dag_reg", "dag_lag", "dag_node", "combo"]
    if not meta["smoothing_class"]:
        names = ["forecast", "factor", "cos", "fw_l1", "adj", "dag_reg", "dag_lag", "dag_node", "combo"]
    for n_, v in zip(names, vals):
        assert_close("val/" + n_, v, d["val/" + n_], 1e-4, 1e-6)


@pytest.mark.parametrize("name", FUSED_SCENARIOS)
def test_forward_and_gc_match_reference(name):
    from oracle.redcliff_oracle import OracleREDCLIFF
    d, meta = load(name)
    m = build(meta)
    m.eval()
    args, kw = ctor_args(meta)
    torch.manual_seed(meta["seed"])
    oracle = OracleREDCLIFF(*args, with_smoothing=meta["smoothing_class"], **kw)
    oracle.eval()
    Xb, Yb = batches(d, meta)[0]
    Lm = max(meta["L"], meta["F"])
    X = Xb[:, :Lm, :].cuda()
    with torch.no_grad():
        x_sim, fpreds, fws, labels = m(X)
    assert_close("x_sim", x_sim.cpu().numpy(), d["eval/x_sim"], RTOL, 1e-5)
    assert_close("w", fws[0].cpu().numpy(), d["eval/w"], RTOL, 1e-5)
    assert_close("labels0", labels[0].cpu().numpy(), d["eval/labels0"], RTOL, 1e-5)
    for k, fp in enumerate(fpreds):
        assert_close("fpred%d" % k, fp.cpu().numpy(), d["eval/fpred%d" % k], RTOL, 1e-5)
    for key in [k for k in d.files if k.startswith("eval/gc/")]:
        _, _, mode, ign, comb = key.split("/")
        gcs = m.GC(mode, X=X, threshold=False, ignore_lag=ign == "ign1", combine_wavelet_representations=comb == "comb1")
        arr = np.stack([np.stack([g.detach().cpu().numpy() for g in row]) for row in gcs])
        assert_close(key, arr, d[key], RTOL, 1e-5)
        # threshold=True thresholds each factor / embedder graph before weighting (cmlp.py:201-202)
        thr = m.GC(mode, X=X, threshold=True, ignore_lag=ign == "ign1", combine_wavelet_representations=comb == "comb1")
        tarr = np.stack([np.stack([g.detach().cpu().numpy() for g in row]) for row in thr])
        with torch.no_grad():
            othr = oracle.GC(mode, X=Xb[:, :Lm, :], threshold=True, ignore_lag=ign == "ign1",
                             combine_wavelet_representations=comb == "comb1")
        oarr = np.stack([np.stack([g.numpy() for g in row]) for row in othr])
        assert_close(key + "/thresholded", tarr, oarr, RTOL, 1e-5)


def test_train_mode_forward_updates_bn_like_reference():
    d, meta = load("dgcnn_c1")
    m = build(meta)
    m.train()
    Xb, _ = batches(d, meta)[0]
    with torch.no_grad():
        x_sim, _, fws, _ = m(Xb[:, :max(meta["L"], meta["F"]), :].cuda())
    assert_close("train x_sim", x_sim.cpu().numpy(), d["train_fwd/x_sim"], RTOL, 1e-5)
    assert_close("train w", fws[0].cpu().numpy(), d["train_fwd/w"], RTOL, 1e-5)
    assert int(m.factor_score_embedder.dgcnn.dgcnn.BN1.num_batches_tracked) == 1


def test_cmlp_gc_prox_forward_match_reference():
    import redcliff_amd
    d, _ = load("cmlp_prox")
    torch.manual_seed(3)
    net = redcliff_amd.cMLP(5, 4, [6]).cuda()
    for ign in (0, 1):
        # a graph tensor, as the reference's torch.norm of the weights (models/cmlp.py:162-166)
        assert_close("gc", net.GC(threshold=False, ignore_lag=bool(ign)).detach().cpu().numpy(), d["gc/ign%d" % ign], 1e-5,
                     1e-6)
        np.testing.assert_array_equal(net.GC(threshold=True, ignore_lag=bool(ign)).cpu().numpy(), d["gct/ign%d" % ign])
    with torch.no_grad():
        y = net(torch.from_numpy(d["fwd/X"]).cuda())
    assert_close("fwd", y.cpu().numpy(), d["fwd/Y"], 1e-5, 1e-6)
    for pen in ("GL", "GSGL", "H"):
        n2 = copy.deepcopy(net)
        n2.perform_prox_update_on_GC_weights(0.9, 0.5, pen)
        want = state(d, "prox_" + pen)
        for k, v in n2.state_dict().items():
            assert_close("prox_%s/%s" % (pen, k), v.cpu().numpy(), want[k], 1e-5, 1e-6)


# --------------------------------------------------------------------------- vs the oracle at real sizes
CONFIGS = {
    # configs[0] C1: p=10, L=gen_lag=5, K=2, h=25, DGCNN F=16 / 3 layers / 100 hidden, B=128
    "C1": dict(p=10, L=5, K=2, nsup=2, h=25, F=16, n=3, H=100, B=128, T=100, label_T=100),
    # C1 north-star ratio config: p=10, L=5, K=4, h=25, DGCNN F=16 / 3 layers / 100 hidden, B=128
    "C1K4": dict(p=10, L=5, K=4, nsup=4, h=25, F=16, n=3, H=100, B=128, T=100, label_T=100),
    # C2 D4IC-shaped: p=10, L=4, K=4, h=100, F=20, 2 layers, 30 hidden, labels (N, K, 1), T=21
    "C2": dict(p=10, L=4, K=4, nsup=4, h=100, F=20, n=2, H=30, B=128, T=21, label_T=1),
    # C4 TST-shaped: p=12, L=4, K=9 (3 supervised), h=25, F=16, 3 layers, 100 hidden, T=150
    "C4": dict(p=12, L=4, K=9, nsup=3, h=25, F=16, n=3, H=100, B=128, T=150, label_T=150),
}
# The reference's grid-search shape classes beyond the published single configs.
# TST grid (train/REDCLIFF_S_CMLP_tst100hzRerun1024AvgReg_gsSmooth1.py:302-303): embed_lag {16, 32, 64} x
# graph-conv layers {2, 3} at the TST model (C4 is (16, 3)); Lmax = embed_lag, so the windows hold
# embed_lag + 1 steps of the 150-step recordings.
GRID_TST = dict(("TST_l%d_n%d" % (F, n), dict(CONFIGS["C4"], F=F, n=n)) for F, n in ((16, 2), (32, 2), (32, 3), (64, 2),
                                                                                    (64, 3)))
# synthetic grid (train/REDCLIFF_S_CMLP_synSysInnovGauss1030_BSCgsSmooth3Parsim.py:140-1131, cached args: gen_lag 4,
# h 25, DGCNN 16 / 3 / 100; K = nsup = numF, p = numN): its extreme classes -- K = 1 (no cosine pairs),
# p = 3 (ADJ_L1 / sqrt(8)), K = 10 on 6 channels, K = 1 on 12
GRID_SYN = dict(("SYN_K%d_p%d" % (K, p), dict(p=p, L=4, K=K, nsup=K, h=25, F=16, n=3, H=100, B=128, T=100, label_T=100))
                for K, p in ((1, 3), (2, 3), (10, 6), (1, 12)))
GRID_CLASSES = dict(GRID_TST, **GRID_SYN)
# C5 stress: p=64, L=20, K=8, h=25, F=64, 3 layers, 100 hidden
C5 = dict(p=64, L=20, K=8, nsup=8, h=25, F=64, n=3, H=100, B=128, T=128, label_T=128)


def oracle_and_hip(cfg, seed=0):
    from oracle.redcliff_oracle import OracleREDCLIFF, reference_coeffs
    import redcliff_amd
    coeff = reference_coeffs(cfg["K"], cfg["p"])
    eargs = [("num_features_per_node", cfg["F"]), ("num_graph_conv_layers", cfg["n"]),
             ("num_hidden_nodes", cfg["H"]), ("sigmoid_eccentricity_coeff", 10.0)]
    args = (cfg["p"], cfg["L"], [cfg["h"]], cfg["F"], [0], cfg["L"], 1, cfg["K"], cfg["nsup"], coeff, False, "DGCNN",
            eargs, "conditional_factor_fixed_embedder", "apply_factor_weights_after_sim_completion")
    kw = dict(num_sims=1, training_mode="pretrain_embedder_then_acclimate_factors_then_combined",
              num_pretrain_epochs=1, num_acclimation_epochs=1)
    torch.manual_seed(seed)
    o = OracleREDCLIFF(*args, **kw)
    torch.manual_seed(seed)
    m = redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing(*args, **kw).cuda()
    return o, m


def synth(cfg, N, seed):
    rng = np.random.RandomState(seed)
    X = rng.randn(N, cfg["T"], cfg["p"]).astype(np.float32)
    for t in range(2, cfg["T"]):
        X[:, t] += 0.4 * X[:, t - 1] - 0.2 * X[:, t - 2]
    X /= X.std()
    if cfg["label_T"] == 1:
        Y = np.zeros((N, cfg["K"], 1), np.float32)
        Y[np.arange(N), rng.randint(0, cfg["K"], N), 0] = 10.0
    else:
        Y = np.zeros((N, cfg["K"], cfg["label_T"]), np.float32)
        Y[np.arange(N), rng.randint(0, cfg["K"], N), :] = 1.0
    return torch.from_numpy(X), torch.from_numpy(Y)


@pytest.mark.parametrize("cname,path", [(c, "auto") for c in CONFIGS] + [("C1", "mfma"), ("C1K4", "mfma"), ("C4", "mfma"),
                                                                        ("C2", "mfma"), ("C1K4", "embgemm"),
                                                                        ("C2", "embgemm"), ("C2", "embgemm-products")])
def test_published_configs_three_phases_vs_oracle(cname, path, monkeypatch):
    _three_phases_vs_oracle(CONFIGS[cname], cname, path, monkeypatch)


@pytest.mark.parametrize("cname,path", [(c, pth) for c in GRID_CLASSES for pth in ("auto", "packed")])
def test_grid_shape_classes_three_phases_vs_oracle(cname, path, monkeypatch):
    """Every TST-grid shape class and the synthetic grid's extreme classes, on the single-fit default
    path ("auto": the fused vector kernels, the merged / split-lead backward) and on the kernels a
    packed grid runs ("packed": the matrix-core factor chain k_fac_*_s16 and the GEMM-shaped
    embedder with its windowed kernels, REDCLIFF_FAC_PATH=mfma + REDCLIFF_EMB_PATH=gemm) -- the same
    three-phase schedule against the oracle as the published configs."""
    _three_phases_vs_oracle(GRID_CLASSES[cname], cname, path, monkeypatch)


def _three_phases_vs_oracle(cfg, cname, path, monkeypatch):
    """path "mfma" forces the matrix-core factor kernels (rc_factor_mfma.hip, normally chosen
    for p*L >= 256; C2's h=100 runs as four 32-unit hidden blocks per network), "embgemm" the
    GEMM-shaped embedder (rc_embed_gemm.hip, normally chosen for p >= 32 or a packed grid of
    >= 16 replicas; its window-sized products in the windowed kernels for p < 32),
    "embgemm-products" the same with those products as batched GEMMs (REDCLIFF_EMB_WIN=0, the
    p >= 32 form) onto the published shapes."""
    if path == "mfma":
        monkeypatch.setenv("REDCLIFF_FAC_PATH", path)
    elif path == "packed":
        monkeypatch.setenv("REDCLIFF_FAC_PATH", "mfma")
        monkeypatch.setenv("REDCLIFF_EMB_PATH", "gemm")
    elif path.startswith("embgemm"):
        monkeypatch.setenv("REDCLIFF_EMB_PATH", "gemm")
        if path == "embgemm-products":
            monkeypatch.setenv("REDCLIFF_EMB_WIN", "0")
    o, m = oracle_and_hip(cfg)
    X, Y = synth(cfg, 2 * cfg["B"] + 40, seed=5)
    B = cfg["B"]
    bs = [(X[i:i + B], Y[i:i + B]) for i in range(0, X.shape[0], B)]
    from oracle.redcliff_oracle import make_optimizers
    oA, oB = make_optimizers(o, 5e-4, 1e-4, 1e-4, 5e-4, 1e-4, 1e-4)
    hA, hB = make_optimizers(m, 5e-4, 1e-4, 1e-4, 5e-4, 1e-4, 1e-4)
    for epoch in (0, 1, 2):
        for bi, (Xb, Yb) in enumerate(bs):
            o.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
            m.batch_update(epoch, bi, Xb, Yb, hA, hB, 1)
    want = dict((k, v.detach().numpy()) for k, v in o.state_dict().items() if not k.startswith("gen_model."))
    compare_state(cname, m, want, rtol=2e-4, atol=5e-6)
    # losses / GC estimates on held-out windows
    Xv, Yv = synth(cfg, 64, seed=9)
    ov = o.validate([(Xv, Yv)])
    hist = [[] for _ in range(5)]
    hv = m.validate_training([(Xv, Yv)], 1, cfg["p"], *hist)
    for i, k in enumerate(["forecast", "factor", "cos", "fw_l1", "smooth", "adj"]):
        assert_close("val/" + k, hv[i], ov[k], 1e-4, 1e-6)
    o.eval()
    m.eval()
    Lm = max(cfg["L"], cfg["F"])
    with torch.no_grad():
        go = o.GC("conditional_factor_fixed_embedder", X=Xv[:40, :Lm], threshold=False, ignore_lag=False)
        gm = m.GC("conditional_factor_fixed_embedder", X=Xv[:40, :Lm].cuda(), threshold=False, ignore_lag=False)
    a = np.stack([np.stack([g.numpy() for g in row]) for row in go])
    b = np.stack([np.stack([g.cpu().numpy() for g in row]) for row in gm])
    assert_close("GC", b, a, 1e-4, 1e-5)
    np.testing.assert_array_equal(b > 0, a > 0)


def _factor_unit(tag, idx):
    """The hidden unit (k, j, u) a factor-network entry belongs to -- row u of layer-0 W0 (h, p, L),
    b0[u], output weight W1[0, u, 0] -- or None (b1, embedder tensors): a unit's ReLU gate is ONE
    discrete decision per window, and a gate that falls the other way moves the whole unit's
    Adam update."""
    m = re.match(r"factors\.(\d+)\.networks\.(\d+)\.layers\.(\d)\.(weight|bias)$", tag)
    if not m:
        return None
    k, j, layer, kind = int(m.group(1)), int(m.group(2)), int(m.group(3)), m.group(4)
    if layer == 0:
        return (k, j, int(idx[0]))
    if kind == "weight":
        return (k, j, int(idx[1]))
    return None


def test_stress_config_error_budget_vs_fp64():
    """C5 (BASELINE configs[4]): p=64, L=20, K=8, B=128 -- the pretrain -> acclimate -> combined
    schedule with TWO batches per phase (six Adam steps), judged against the SAME oracle run in
    float64 from the same initial values and inputs.

    Reference fp32 variability: three fp32 realisations of the oracle -- the batches as given,
    every batch's rows permuted (another order of the batch reductions), and the factor
    contraction's input channels permuted (another fp32 order of the p*L = 1280-term hidden
    pre-activations, which is what the HIP path's matrix-core k-order changes; the row
    permutation does not touch it) -- and a float64 run with every near-tie decision taken the
    other way (c5_oracle_runs.FlipNearTies).  Four fp32 realisations in all: the HIP path and the
    three oracle runs.  The five oracle trajectories run side by side in worker processes
    (tests/c5_oracle_runs.py) while the GPU runs the HIP path.  For each realisation Z and every
    parameter / buffer entry:

        |Z - fp64| <= 3 max_{other realisations O} |O - fp64| + |fp64_tieflip - fp64| + 1e-4 |fp64| + 1e-7

    Outliers are counted per DECISION: the entries of one factor hidden unit (its W0 row, b0 and
    W1 entries) move together when that unit's ReLU gate falls the other way for some window, so
    a unit with any outlier counts once.  A GATE-FLIP unit is an outlier unit whose float64 gate
    is a near-tie: for some window of some training step its pre-activation came within 1e-6 (the
    fp32 resolution of the p*L = 1280-term contraction, FlipNearTies' band) of zero relative to its
    network's largest (c5_oracle_runs.GateMargins) -- the HIP path's contraction is one fmaf chain
    on the matrix cores, the CPU's is vectorised, so its fp32 error is its own and such gates can
    fall either way.  Required:
      * at most 1e-3 of the 12,800 units are gate-flip units, and inside them no entry is further
        than 2 lr (two Adam steps) from float64;
      * every other outlier entry is fp32 tail: at most max(reference runs' tail entries + 2, one
        per million) of them, none exceeding 2x the reference runs' worst excess or 1e-2 lr;
      * losses within |oracle_fp32 - fp64| + 1e-4 |fp64|;
      * GC extraction on the HIP model's own final parameters within 1e-4 relative of the float64
        oracle's on the same parameters, with identical thresholded graphs.
    Thresholded graphs of the TRAJECTORIES (lag-free conditional GC of 8 validation windows,
    262,144 entries):
      * the HIP graph equals the fp32 oracle's own graph wherever the oracle's realisations (the
        three fp32 runs, float64, tie-flipped float64) agree on the sign; every disagreement lies
        at an entry where they disagree among themselves;
      * it equals the float64 trajectory's graph wherever float64 decides the sign at fp32
        resolution (|g64| above 3x the spread of the reference's fp32 runs and of the tie run);
      * the entries NOT so decided are at most 5e-5 of all (13 of 262,144; the round-2 run with
        one batch per phase had 6), so the exclusion cannot hide a systematic error.
    Why not "every entry inside |oracle_fp32 - fp64|": a step takes 0.8 M embedder gates,
    0.8 M factor gates and 67 M adjacency-L1 signs, so some sit within fp32 rounding of zero, and
    an Adam update eps-normalised from a gradient that nearly cancels amplifies rounding by
    lr/eps; round 3's first two-batches-per-phase run (window-permuted realisations only) put
    836 of the HIP path's 842 outlier entries in ONE hidden unit (factors.4.networks.2, u=10),
    i.e. one gate decision."""
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor
    import c5_oracle_runs as C5R
    cfg = dict(C5, B=128)
    NB = 2
    lr = C5R.LR
    TIE = 1e-6  # fp32 tie band of a hidden pre-activation (c5_oracle_runs.FlipNearTies tau_factor)
    X, Y = synth(cfg, NB * cfg["B"], seed=5)
    Xv, Yv = synth(cfg, 40, seed=9)
    kinds = ["fp32", "perm1", "chperm1", "fp64", "fp64flip"]
    with ProcessPoolExecutor(len(kinds), mp_context=mp.get_context("spawn")) as ex:
        futs = dict((k, ex.submit(C5R.trajectory, k, cfg, X.numpy(), Y.numpy(), Xv.numpy(), Yv.numpy(), NB))
                    for k in kinds)
        _, m = oracle_and_hip(cfg)
        hA, hB = make_opts(m, lr, lr)
        B = cfg["B"]
        for epoch in (0, 1, 2):
            for bi in range(NB):
                m.batch_update(epoch, bi, X[bi * B:(bi + 1) * B], Y[bi * B:(bi + 1) * B], hA, hB, 1)
        hv = m.validate_training([(Xv, Yv)], 1, cfg["p"], *[[] for _ in range(5)])
        m.eval()
        Lm = max(cfg["L"], cfg["F"])
        Xg = Xv[:8, :Lm]
        with torch.no_grad():
            g_hip = C5R.gc_of(m, Xg.cuda())
        got = dict((k, v.detach().cpu().numpy()) for k, v in m.state_dict().items() if not k.startswith("gen_model."))
        res = dict((k, f.result(timeout=600)) for k, f in futs.items())
    print("near-tie decisions flipped in the float64 tie run: %s" % res["fp64flip"]["flipped"])
    runs = [res[k] for k in ("fp32", "perm1", "chperm1")]
    r64, r64f = res["fp64"], res["fp64flip"]
    nreal = 1 + len(runs)            # realisation 0 is the HIP path
    units = [set() for _ in range(nreal)]
    outl = [[] for _ in range(nreal)]  # (tag, flat index, excess, unit, fp64 value, this run's value)
    n_entries = [0]

    def envelope(tag, reals, x, t):
        """reals: [HIP, oracle runs...] arrays; x fp64, t tie-flipped fp64."""
        dev = np.stack([np.abs(np.asarray(r, np.float64) - x) for r in reals])
        n_entries[0] += x.size
        base = np.abs(t - x) + 1e-4 * np.abs(x) + 1e-7
        for z in range(nreal):
            others = np.delete(dev, z, axis=0).max(axis=0)
            over = dev[z] - (3.0 * others + base)
            for i in np.flatnonzero(over > 0):
                u = _factor_unit(tag, np.unravel_index(i, x.shape))
                if u is not None:
                    units[z].add(u)
                outl[z].append((tag, int(i), float(over.flat[i]), u, float(x.flat[i]),
                                float(np.asarray(reals[z], np.float64).flat[i]), float(dev[z].flat[i])))

    for k in r64["state"]:
        if k.endswith("num_batches_tracked"):
            assert int(got[k]) == int(r64["state"][k]) == int(runs[0]["state"][k]), k
            continue
        envelope(k, [got[k]] + [r_["state"][k] for r_ in runs], r64["state"][k].astype(np.float64),
                 r64f["state"][k].astype(np.float64))
    margin = r64["gate_margin"]  # (K, p, h): min over steps / windows of |z| / max|z| in float64
    print("float64 gate margins of the outlier units: HIP %s" % ["%s %.2e" % (u_, margin[u_]) for u_ in sorted(units[0])])
    print("units with a float64 gate margin below 1e-6 / 1e-4: %d / %d of %d"
          % (int((margin <= TIE).sum()), int((margin <= 1e-4).sum()), margin.size))
    # a gate-flip unit: an outlier unit whose float64 gate came within the fp32 tie band; every
    # other outlier entry (single entries of units whose gate never came that close, embedder
    # tensors) is fp32 tail and is held to the tail rule below
    gate = [set(u_ for u_ in units[z] if margin[u_] <= TIE) for z in range(nreal)]
    rest = [[o for o in outl[z] if o[3] not in gate[z]] for z in range(nreal)]
    worst_rest = [max([o[2] for o in rest[z]], default=0.0) for z in range(nreal)]
    in_units = [o for o in outl[0] if o[3] in gate[0]]
    print("gate-flip units: HIP %s, oracle runs %s" % (sorted(gate[0]), [len(g_) for g_ in gate[1:]]))
    print("outlier entries outside them: HIP %d (worst excess %.3e), oracle runs %s (worst %s)"
          % (len(rest[0]), worst_rest[0], [len(r_) for r_ in rest[1:]], ["%.3e" % w for w in worst_rest[1:]]))
    for o in sorted(rest[0], key=lambda o: -o[2])[:12]:
        print("  HIP tail entry %s[%d]: excess %.3e, |HIP - fp64| %.3e (%.3f lr), fp64 %.6e, unit %s"
              % (o[0], o[1], o[2], o[6], o[6] / lr, o[4], o[3]))
    if in_units:
        print("HIP gate-flip units: %d entries, largest |HIP - fp64| %.3e (= %.2f lr)"
              % (len(in_units), max(o[6] for o in in_units), max(o[6] for o in in_units) / lr))
    assert len(gate[0]) <= 1e-3 * margin.size, "too many gate-flip units: %d" % len(gate[0])
    assert all(o[6] <= 2.0 * lr for o in in_units), "a gate-flip unit moved further than two Adam steps"
    assert len(rest[0]) <= max(max(len(r_) for r_ in rest[1:]) + 2, 1e-6 * n_entries[0]), \
        "HIP path's fp32 tail beyond the reference's"
    assert worst_rest[0] <= max(2.0 * max(worst_rest[1:]), 1e-2 * lr), "HIP path's worst excess beyond the reference's"
    for i, k in enumerate(["forecast", "factor", "cos", "fw_l1", "smooth", "adj"]):
        ov, ov64 = runs[0]["val"][k], r64["val"][k]
        assert abs(hv[i] - ov64) <= abs(ov - ov64) + 1e-4 * abs(ov64) + 1e-7, (k, hv[i], ov, ov64)
    # GC extraction on the SAME parameters: the HIP model's final state loaded into the float64
    # oracle (the trajectory is judged above; this isolates the GC computation), 1e-4 relative
    o64h = C5R.build_oracle(cfg).double()
    o64h.load_state_dict(dict((k, v.detach().cpu().double() if v.is_floating_point() else v.detach().cpu())
                              for k, v in m.state_dict().items()))
    o64h.eval()
    with torch.no_grad(), C5R.Float64Default():
        g64h = C5R.gc_of(o64h, Xg.double())
    gexcess = np.abs(g_hip - g64h) - (1e-4 * np.abs(g64h) + 1e-6 * np.abs(g64h).max())
    print("GC on the HIP parameters vs float64: max |err| %.3e, worst excess over 1e-4 rel %.3e"
          % (np.abs(g_hip - g64h).max(), gexcess.max()))
    assert gexcess.max() <= 0, "GC extraction differs from float64 on the same parameters"
    np.testing.assert_array_equal(g_hip > 0, g64h > 0)
    # ---- thresholded graphs of the trajectories
    g_runs = [r_["gc"] for r_ in runs]
    g64, g64f = r64["gc"], r64f["gc"]
    signs = np.stack([g > 0 for g in g_runs + [g64, g64f]])
    contested = signs.any(axis=0) & ~signs.all(axis=0)       # the reference's realisations disagree
    d_or = (g_hip > 0) != (g_runs[0] > 0)
    print("HIP vs fp32 oracle graph: %d differing entries, %d contested among the oracle's realisations; "
          "differing AND uncontested: %d" % (int(d_or.sum()), int(contested.sum()), int((d_or & ~contested).sum())))
    assert not (d_or & ~contested).any(), "HIP graph differs from the fp32 oracle's where the reference agrees"
    band = 3.0 * np.max(np.stack([np.abs(g - g64) for g in g_runs] + [np.abs(g64f - g64)]), axis=0) \
        + 1e-6 * np.abs(g64).max()
    decided = np.abs(g64) > band
    n_und = int((~decided).sum())
    print("trajectory graph entries decided at fp32 resolution: %d / %d (undecided %d)"
          % (int(decided.sum()), decided.size, n_und))
    assert n_und <= 5e-5 * decided.size, "too many entries undecided at fp32 resolution: %d" % n_und
    np.testing.assert_array_equal((g_hip > 0)[decided], (g64 > 0)[decided])


def test_fit_trace_matches_reference():
    import redcliff_amd
    d, meta = load("fit_trace")
    args = (meta["p"], meta["L"], [meta["h"]], meta["F"], [0], meta["L"], 1, meta["K"], meta["nsup"], meta["coeff"],
            False, "DGCNN", [("num_features_per_node", meta["F"]), ("num_graph_conv_layers", meta["n"]),
                             ("num_hidden_nodes", meta["H"]), ("sigmoid_eccentricity_coeff", 10.0)],
            meta["gc_mode"], meta["fwd_mode"])
    torch.manual_seed(meta["seed"])
    m = redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing(*args, num_sims=1, training_mode=meta["training_mode"],
                                                        num_pretrain_epochs=meta["pre"],
                                                        num_acclimation_epochs=meta["acc"]).cuda()
    B = meta["B"]
    X, Y, Xv, Yv = [torch.from_numpy(d[k]) for k in ("X", "Y", "Xv", "Yv")]
    train = [(X[i:i + B], Y[i:i + B]) for i in range(0, len(X), B)]
    val = [(Xv[i:i + B], Yv[i:i + B]) for i in range(0, len(Xv), B)]
    true_gc = [d["true_gc%d" % k] for k in range(meta["K"])]
    oA, oB = make_opts(m, 5e-4, 5e-4)
    m.fit(None, train, oA, oB, meta["L"], 1, 1, meta["max_iter"], val, lookback=1, check_every=1, verbose=0,
          GC=true_gc, stopping_criteria_forecast_coeff=10., stopping_criteria_factor_coeff=100.,
          stopping_criteria_cosSim_coeff=1.)
    h = m.fit_history
    for k in ("avg_forecasting_loss", "avg_factor_loss", "avg_factor_cos_sim_penalty", "avg_fw_l1_penalty",
              "avg_adj_penalty", "avg_combo_loss"):
        assert_close(k, np.asarray(h[k]), d["hist/" + k], 1e-4, 1e-6)
    assert h["best_it"] == int(d["hist/best_it"])
    for sf in range(meta["K"]):
        np.testing.assert_allclose(h["f1score_histories"][0.0][sf], d["hist/f1_%d" % sf], rtol=0, atol=1e-6)
    compare_state("final", m, state(d, "final"), rtol=2e-4, atol=5e-6)
    m.eval()
    with torch.no_grad():
        gcs = m.GC(meta["gc_mode"], X=val[0][0][:, :max(meta["L"], meta["F"])].cuda(), threshold=False,
                   ignore_lag=False, combine_wavelet_representations=True)
    arr = np.stack([np.stack([g.cpu().numpy() for g in row]) for row in gcs])
    assert_close("final_gc", arr, d["final_gc"], 1e-4, 1e-5)
    from redcliff_amd.metrics import get_f1_score
    f1 = np.asarray([[get_f1_score(g.sum(axis=2) / np.max(g.sum(axis=2)), true_gc[k].sum(axis=2))
                      for k, g in enumerate(row)] for row in arr])
    np.testing.assert_array_equal(f1, d["f1"])


@pytest.mark.parametrize("name", ["dgcnn_d4ic", "dgcnn_c1"])
def test_eval_pipeline_f1_identical_to_oracle(name):
    """SURVEY 8(f) row 3 on the GPU model: eval_utils.get_model_gc_estimates (primary GC mode,
    one sample, lagged, unthresholded) from the HIP model vs the oracle, then the
    system-level statistics and the optimal-F1 thresholded graphs -- F1 and graphs must be
    IDENTICAL (north_star), the continuous statistics within 1e-4 relative."""
    from oracle.redcliff_oracle import OracleREDCLIFF
    from redcliff_amd import evaluation as E
    d, meta = load(name)
    m = build(meta)
    m.eval()
    args, kw = ctor_args(meta)
    torch.manual_seed(meta["seed"])
    oracle = OracleREDCLIFF(*args, with_smoothing=meta["smoothing_class"], **kw)
    oracle.eval()
    Xb, _ = batches(d, meta)[0]
    Lm = max(meta["L"], meta["F"])
    K, p = meta["K"], meta["p"]
    got = E.get_model_gc_estimates(m, "REDCLIFF_S_CMLP", K, X=Xb[:1, :Lm, :].cuda())
    with torch.no_grad():
        want = E.get_model_gc_estimates(oracle, "REDCLIFF_S_CMLP", K, X=Xb[:1, :Lm, :])
    assert len(got) == len(want) == K
    for k in range(K):
        assert_close("gc%d" % k, got[k], want[k], RTOL, 1e-5)
    rng = np.random.RandomState(3)
    trus = []
    for _ in range(K):
        t = np.zeros((p, p, got[0].shape[2]))  # sorting compares flattened graphs: same lag count
        t[..., 0] = rng.rand(p, p) < 0.3
        t[0, 1, 0], t[1, 0, 0] = 1.0, 0.0
        trus.append(t)
    with np.errstate(all="ignore"):
        sg = E.system_level_factor_stats(got, trus, sort_unsupervised_ests=True)
        sw = E.system_level_factor_stats(want, trus, sort_unsupervised_ests=True)
    for key in ("cos_sim", "mse", "roc_auc", "T_cos_sim", "dir_deltacon0", "deltaffinity"):
        assert_close(key, sg[key], sw[key], 1e-4, 1e-6)
    rg = E.batched_graph_f1(np.stack(got), np.stack(trus))
    rw = E.batched_graph_f1(np.stack(want), np.stack(trus))
    assert np.array_equal(rg["f1"], rw["f1"]), (rg["f1"], rw["f1"])
    assert np.array_equal(rg["graphs"], rw["graphs"])
