"""Pin the CPU oracle (oracle/redcliff_oracle.py) against golden vectors from the reference.

CPU-only.  Fixtures are produced by tests/golden/make_golden.py, which runs the reference
code itself in the build container; scenarios using the DGCNN embedder are pinned only
up to the torcheeg 1.1.3 restatement (oracle/torcheeg_dgcnn.py).
"""
import copy

import numpy as np
import pytest
import torch

from golden_io import SCENARIOS, assert_close, batches, ctor_args, load, state
from oracle.redcliff_oracle import OracleREDCLIFF, f1_score_graph, OCMLP

# identical op structure to the reference -> only fp32 re-association noise is allowed
RTOL, ATOL = 2e-5, 2e-6


def build_oracle(meta):
    args, kw = ctor_args(meta)
    torch.manual_seed(meta["seed"])
    return OracleREDCLIFF(*args, with_smoothing=meta["smoothing_class"], **kw).float()


def compare_state(tag, model, want, rtol=RTOL, atol=ATOL):
    got = dict((k, v.detach().numpy()) for k, v in model.state_dict().items() if not k.startswith("gen_model."))
    assert set(got) == set(want), "%s: key sets differ: %s" % (tag, sorted(set(got) ^ set(want)))
    for k in want:
        assert_close("%s/%s" % (tag, k), got[k], want[k], rtol, atol)


@pytest.mark.parametrize("name", SCENARIOS)
def test_init_matches_reference_rng_order(name):
    d, meta = load(name)
    m = build_oracle(meta)
    compare_state("init", m, state(d, "init"), rtol=0, atol=0)


@pytest.mark.parametrize("name", SCENARIOS)
def test_eval_forward_gc_loss(name):
    d, meta = load(name)
    m = build_oracle(meta)
    m.eval()
    bs = batches(d, meta)
    Xb, Yb = bs[0]
    Lm = max(meta["L"], meta["F"])
    with torch.no_grad():
        x_sim, fpreds, fws, labels = m(Xb[:, :Lm, :])
        assert_close("x_sim", x_sim.numpy(), d["eval/x_sim"], RTOL, ATOL)
        assert_close("w", fws[0].numpy(), d["eval/w"], RTOL, ATOL)
        assert_close("labels0", labels[0].numpy(), d["eval/labels0"], RTOL, ATOL)
        for key in [k for k in d.files if k.startswith("eval/gc/")]:
            _, _, mode, ign, comb = key.split("/")
            gcs = m.GC(mode, X=Xb[:, :Lm, :], threshold=False, ignore_lag=ign == "ign1",
                       combine_wavelet_representations=comb == "comb1")
            arr = np.stack([np.stack([g.numpy() for g in row]) for row in gcs])
            assert_close(key, arr, d[key], RTOL, ATOL)
        tgt = Xb[:, Lm:Lm + meta["S"], :]
        for flag in ("combined", "emb", "fac"):
            combo, terms = m.compute_loss(Xb[:, :meta["F"], :], x_sim, tgt, labels, Yb, meta["gc_mode"],
                                          embedder_pretrain_loss=flag == "emb", factor_pretrain_loss=flag == "fac")
            assert_close("combo/" + flag, float(combo), d["eval/loss/%s/combo" % flag], RTOL, 1e-5)
            for i, t in enumerate(terms):
                want = d["eval/loss/%s/t%d" % (flag, i)]
                if np.isnan(want):
                    assert t is None
                else:
                    assert_close("term%d/%s" % (i, flag), float(t), want, RTOL, 1e-5)


@pytest.mark.parametrize("name", SCENARIOS)
def test_train_mode_forward(name):
    d, meta = load(name)
    m = build_oracle(meta)
    m.train()
    Xb, _ = batches(d, meta)[0]
    with torch.no_grad():
        x_sim, _, fws, _ = m(Xb[:, :max(meta["L"], meta["F"]), :])
    assert_close("train x_sim", x_sim.numpy(), d["train_fwd/x_sim"], RTOL, ATOL)
    assert_close("train w", fws[0].numpy(), d["train_fwd/w"], RTOL, ATOL)


@pytest.mark.parametrize("name", SCENARIOS)
def test_batch_update_schedule(name):
    d, meta = load(name)
    m = build_oracle(meta)
    oA = torch.optim.Adam(m.gen_model[0].parameters(), lr=meta["lrA"], betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    oB = torch.optim.Adam(m.gen_model[1].parameters(), lr=meta["lrB"], betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    bs = batches(d, meta)
    step = 0
    for epoch in meta["epochs"]:
        for bi, (Xb, Yb) in enumerate(bs):
            m.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
            step += 1
            compare_state("step%d" % step, m, state(d, "step%d" % step), rtol=1e-4, atol=1e-5)
    assert step == int(d["nsteps"])
    vals = m.validate(bs)
    for k in ("forecast", "factor", "cos", "fw_l1", "adj", "combo"):
        assert_close("val/" + k, vals[k], d["val/" + k], 1e-4, 1e-5)


def test_cmlp_gc_and_prox():
    d, _ = load("cmlp_prox")
    torch.manual_seed(3)
    net = OCMLP(5, 4, [6])
    init = state(d, "init")
    for k, v in net.state_dict().items():
        assert_close("init/" + k, v.numpy(), init[k], 0, 0)
    for ign in (0, 1):
        assert_close("gc", net.GC(threshold=False, ignore_lag=bool(ign)).detach().numpy(), d["gc/ign%d" % ign], 1e-6, 1e-7)
        assert (net.GC(threshold=True, ignore_lag=bool(ign)).numpy() == d["gct/ign%d" % ign]).all()
    with torch.no_grad():
        assert_close("fwd", net(torch.from_numpy(d["fwd/X"])).numpy(), d["fwd/Y"], 1e-6, 1e-6)
    for pen in ("GL", "GSGL", "H"):
        n2 = copy.deepcopy(net)
        n2.prox(0.9, 0.5, pen)
        want = state(d, "prox_" + pen)
        for k, v in n2.state_dict().items():
            assert_close("prox_%s/%s" % (pen, k), v.numpy(), want[k], 1e-6, 1e-7)


def test_fit_trace_f1_metric():
    d, meta = load("fit_trace")
    true = [d["true_gc%d" % k] for k in range(meta["K"])]
    for b, row in enumerate(d["final_gc"]):
        for k, g in enumerate(row):
            s = g.sum(axis=2)
            assert abs(f1_score_graph(s / s.max(), true[k].sum(axis=2)) - d["f1"][b, k]) < 1e-6
