"""Generate golden vectors from the REFERENCE itself (run in the build container only).

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

The reference (/root/reference, read-only) is imported with the two stubs described in
oracle/ref_import.py (empty ``pywt``; torcheeg's DGCNN restated in
oracle/torcheeg_dgcnn.py).  Only data leaves this script: seeded inputs and the
reference's outputs, stored as ``.npz`` (no pickles).  Scenarios cover every
embedder type, both model classes, both forward modes, num_sims 1 and 2, all three
training phases, every valid GC mode and the cMLP proximal steps.

Fixture key conventions (see tests/golden_io.py):
  meta                       JSON string with the constructor arguments / schedule
  X, Y                       the dataset (N, T, p) / labels
  init/<state_dict key>      parameters + buffers right after seeded construction
  eval/...                   eval-mode forward, GC and compute_loss outputs on batch 0
  train_fwd/...              train-mode forward on batch 0 (deep copy, BN batch stats)
  step<i>/<state_dict key>   state after the i-th batch_update of the schedule
  val/<term>                 validate_training averages after the schedule
"""
import copy
import json
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.ref_import import import_reference  # noqa: E402
from oracle.redcliff_oracle import reference_coeffs  # noqa: E402

REF = import_reference()


def _np(t):
    return t.detach().cpu().numpy().copy()


def _sd(prefix, model, out):
    for k, v in model.state_dict().items():
        if not k.startswith("gen_model."):  # gen_model.* aliases duplicate the other keys
            out["%s/%s" % (prefix, k)] = _np(v)


def make_data(N, T, p, K, label_T, seed):
    rng = np.random.RandomState(seed)
    X = rng.randn(N, T, p).astype(np.float32)
    # weak sVAR-like structure so the factors have something to fit
    for t in range(2, T):
        X[:, t] += 0.3 * X[:, t - 1] - 0.1 * X[:, t - 2]
    X = (X - X.mean(axis=(0, 1), keepdims=True)) / X.std(axis=(0, 1), keepdims=True)
    if label_T == 0:
        Y = rng.rand(N, K).astype(np.float32)
    else:
        cls = rng.randint(0, K, size=(N,))
        Y = np.zeros((N, K, label_T), dtype=np.float32)
        Y[np.arange(N), cls, :] = 1.0
        Y += 0.05 * rng.rand(N, K, label_T).astype(np.float32)
    return X.astype(np.float32), Y.astype(np.float32)


def build(cfg):
    torch.manual_seed(cfg["seed"])
    if cfg["emb"] == "DGCNN":
        eargs = [("num_features_per_node", cfg["F"]), ("num_graph_conv_layers", cfg["n"]),
                 ("num_hidden_nodes", cfg["H"]), ("sigmoid_eccentricity_coeff", 10.0)]
    elif cfg["emb"] == "cEmbedder":
        eargs = [("sigmoid_eccentricity_coeff", 10.0), ("lag", cfg["F"]), ("hidden", [cfg["eh"]])]
    else:
        eargs = []
    coeff = reference_coeffs(cfg["K"], cfg["p"], smooth=cfg.get("smooth", 0.0))
    cls = REF.redcliff_smooth.REDCLIFF_S_CMLP_withStateSmoothing if cfg["smoothing_class"] else REF.redcliff.REDCLIFF_S_CMLP
    kw = dict(num_sims=cfg["S"], wavelet_level=cfg.get("wl"), save_path=None, training_mode=cfg["training_mode"],
              num_pretrain_epochs=cfg["pre"], num_acclimation_epochs=cfg["acc"])
    if cfg["smoothing_class"]:
        kw["STATE_SCORE_SMOOTHING_EPSILON"] = 0.0001
    m = cls(cfg["p"], cfg["L"], [cfg["h"]], cfg["F"], [cfg.get("eh", 0)], cfg["L"], 1, cfg["K"], cfg["nsup"], coeff,
            cfg["sigmoid"], cfg["emb"], eargs, cfg["gc_mode"], cfg["fwd_mode"], **kw).float()
    return m, coeff


def valid_gc_modes(cfg):
    modes = ["fixed_factor_exclusive", "conditional_factor_exclusive"]
    if cfg["emb"] in ("cEmbedder", "DGCNN"):
        modes += ["raw_embedder", "fixed_embedder_exclusive", "fixed_factor_fixed_embedder",
                  "conditional_factor_fixed_embedder"]
        if cfg["emb"] == "cEmbedder":
            modes += ["conditional_embedder_exclusive", "fixed_factor_conditional_embedder",
                      "conditional_factor_conditional_embedder"]
    return modes


def record_eval(m, cfg, Xb, Yb, out, prefix):
    Lm = max(cfg["L"], cfg["F"])
    x_sim, fpreds, fws, labels = m(Xb[:, :Lm, :])
    out[prefix + "/x_sim"] = _np(x_sim)
    out[prefix + "/w"] = _np(fws[0])
    out[prefix + "/labels0"] = _np(labels[0])
    if cfg["fwd_mode"] == "apply_factor_weights_after_sim_completion":
        for k, fp in enumerate(fpreds):
            out[prefix + "/fpred%d" % k] = _np(fp)
    if prefix == "eval":
        wl = cfg.get("wl") is not None
        for mode in valid_gc_modes(cfg):
            for ign in (True, False):
                for comb in (False, True):
                    for rank in ((False, True) if wl else (False,)):
                        key = "%s/gc/%s/ign%d/comb%d" % (prefix, mode, int(ign), int(comb)) + ("/rank%d" % rank if wl else "")
                        try:
                            gcs = m.GC(mode, X=Xb[:, :Lm, :], threshold=False, ignore_lag=ign,
                                       combine_wavelet_representations=comb, rank_wavelets=rank)
                        except Exception as e:  # the reference's own failure for this combination
                            if not wl:
                                raise
                            out[key + "/err"] = np.asarray(type(e).__name__)
                            continue
                        out[key] = np.stack([np.stack([_np(g) for g in row]) for row in gcs])
        tgt = Xb[:, Lm:Lm + cfg["S"], :]
        for flag in ("combined", "emb", "fac"):
            combo, terms = m.compute_loss(Xb[:, :cfg["F"], :], x_sim, tgt, labels, Yb, cfg["gc_mode"],
                                          embedder_pretrain_loss=(flag == "emb"),
                                          factor_pretrain_loss=(flag == "fac"))
            out["%s/loss/%s/combo" % (prefix, flag)] = np.asarray(float(combo), dtype=np.float64)
            for i, t in enumerate(terms):
                out["%s/loss/%s/t%d" % (prefix, flag, i)] = np.asarray(np.nan if t is None else float(t), dtype=np.float64)


def run_scenario(name, cfg):
    out = {}
    m, coeff = build(cfg)
    ns = cfg["p"] * (cfg["wl"] + 1) if cfg.get("wl") is not None else cfg["p"]  # wavelet series
    X, Y = make_data(cfg["N"], cfg["T"], ns, cfg["K"], cfg["label_T"], cfg["data_seed"])
    out["X"], out["Y"] = X, Y
    _sd("init", m, out)
    if cfg.get("wl") is not None:  # the ranking masks (plain attributes, not in the state_dict)
        out["wavelet_mask/factor"] = _np(m.factors[0].wavelet_mask)
        if cfg["emb"] == "cEmbedder":
            out["wavelet_mask/embedder"] = _np(m.factor_score_embedder.wavelet_mask)
    B = cfg["B"]
    batches = [(torch.from_numpy(X[i:i + B]), torch.from_numpy(Y[i:i + B])) for i in range(0, cfg["N"], B)]
    # eval-mode probes on a deep copy (BN running stats untouched in the main model)
    probe = copy.deepcopy(m)
    probe.eval()
    with torch.no_grad():
        record_eval(probe, cfg, batches[0][0], batches[0][1], out, "eval")
    probe = copy.deepcopy(m)
    probe.train()
    with torch.no_grad():
        record_eval(probe, cfg, batches[0][0], batches[0][1], out, "train_fwd")
    oA = torch.optim.Adam(m.gen_model[0].parameters(), lr=cfg["lrA"], betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    oB = torch.optim.Adam(m.gen_model[1].parameters(), lr=cfg["lrB"], betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    step = 0
    for epoch in cfg["epochs"]:
        for bi, (Xb, Yb) in enumerate(batches):
            m.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
            step += 1
            _sd("step%d" % step, m, out)
    out["nsteps"] = np.asarray(step)
    hist = [[] for _ in range(5)] if cfg["nsup"] > 0 else [None] * 5
    vals = m.validate_training(batches, 1, ns, *hist)
    names = ["forecast", "factor", "cos", "fw_l1", "smooth", "adj", "dag_reg", "dag_lag", "dag_node", "combo"]
    if not cfg["smoothing_class"]:
        names = ["forecast", "factor", "cos", "fw_l1", "adj", "dag_reg", "dag_lag", "dag_node", "combo"]
    for n_, v in zip(names, vals[:len(names)]):
        out["val/" + n_] = np.asarray(float(v), dtype=np.float64)
    meta = dict(cfg)
    meta["coeff"] = coeff
    out["meta"] = np.asarray(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print("wrote", name, len(out), "arrays")


def run_prox():
    out = {}
    torch.manual_seed(3)
    net = REF.cmlp.cMLP(5, 4, [6])
    _sd("init", net, out)
    for ign in (True, False):
        out["gc/ign%d" % int(ign)] = _np(net.GC(threshold=False, ignore_lag=ign))
        out["gct/ign%d" % int(ign)] = _np(net.GC(threshold=True, ignore_lag=ign))
    X = torch.from_numpy(np.random.RandomState(5).randn(7, 4, 5).astype(np.float32))
    out["fwd/X"] = _np(X)
    out["fwd/Y"] = _np(net(X))
    for pen in ("GL", "GSGL", "H"):
        n2 = copy.deepcopy(net)
        n2.perform_prox_update_on_GC_weights(0.9, 0.5, pen)
        _sd("prox_%s" % pen, n2, out)
    np.savez_compressed(os.path.join(HERE, "cmlp_prox.npz"), **out)
    print("wrote cmlp_prox")


_CAPTURED = {}


def _capture_checkpoint(self, save_dir, it, best_model, *args, **kwargs):
    """Stands in for save_checkpoint (plots + pickles): keeps its arguments in memory."""
    names = ["avg_forecasting_loss", "avg_factor_loss", "avg_factor_cos_sim_penalty", "avg_fw_l1_penalty",
             "avg_fw_smoothing_penalty", "avg_adj_penalty", "avg_dagness_reg_loss", "avg_dagness_lag_loss",
             "avg_dagness_node_loss", "avg_combo_loss", "best_loss", "best_it", "f1score_histories"]
    _CAPTURED.clear()
    _CAPTURED.update(dict(zip(names, [copy.deepcopy(a) for a in args[:len(names)]])))
    _CAPTURED["epoch"] = it


def run_fit():
    """A short reference fit() trace (C1-shaped, tiny)."""
    cfg = dict(seed=21, emb="DGCNN", p=5, L=2, K=2, nsup=2, h=6, F=3, n=2, H=4, S=1, sigmoid=False,
               smoothing_class=True, gc_mode="conditional_factor_fixed_embedder",
               fwd_mode="apply_factor_weights_after_sim_completion",
               training_mode="pretrain_embedder_then_acclimate_factors_then_combined", pre=1, acc=1,
               N=48, T=10, label_T=10, data_seed=11, B=16)
    m, coeff = build(cfg)
    ns = cfg["p"] * (cfg["wl"] + 1) if cfg.get("wl") is not None else cfg["p"]  # wavelet series
    X, Y = make_data(cfg["N"], cfg["T"], ns, cfg["K"], cfg["label_T"], cfg["data_seed"])
    Xv, Yv = make_data(32, cfg["T"], cfg["p"], cfg["K"], cfg["label_T"], 12)
    B = cfg["B"]
    train = [(torch.from_numpy(X[i:i + B]), torch.from_numpy(Y[i:i + B])) for i in range(0, len(X), B)]
    val = [(torch.from_numpy(Xv[i:i + B]), torch.from_numpy(Yv[i:i + B])) for i in range(0, len(Xv), B)]
    rng = np.random.RandomState(7)
    true_gc = [(rng.rand(cfg["p"], cfg["p"], 2) > 0.6).astype(np.float64) for _ in range(cfg["K"])]
    out = {"X": X, "Y": Y, "Xv": Xv, "Yv": Yv}
    for i, g in enumerate(true_gc):
        out["true_gc%d" % i] = g
    _sd("init", m, out)
    oA = torch.optim.Adam(m.gen_model[0].parameters(), lr=5e-4, betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    oB = torch.optim.Adam(m.gen_model[1].parameters(), lr=5e-4, betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    max_iter = 8
    _CAPTURED.clear()
    cls = type(m)
    orig = cls.save_checkpoint
    cls.save_checkpoint = _capture_checkpoint
    try:
        with tempfile.TemporaryDirectory() as d:
            m.fit(d, train, oA, oB, cfg["L"], 1, 1, max_iter, val, lookback=1, check_every=1, verbose=0, GC=true_gc,
                  stopping_criteria_forecast_coeff=10., stopping_criteria_factor_coeff=100.,
                  stopping_criteria_cosSim_coeff=1.)
    finally:
        cls.save_checkpoint = orig
    meta = dict(_CAPTURED)
    _sd("final", m, out)
    for k in ("avg_forecasting_loss", "avg_factor_loss", "avg_factor_cos_sim_penalty", "avg_fw_l1_penalty",
              "avg_fw_smoothing_penalty", "avg_adj_penalty", "avg_combo_loss"):
        out["hist/" + k] = np.asarray(meta[k], dtype=np.float64)
    out["hist/best_it"] = np.asarray(meta["best_it"])
    out["hist/last_epoch"] = np.asarray(meta["epoch"])
    out["hist/best_loss"] = np.asarray(float(meta["best_loss"]))
    for sf in range(cfg["K"]):
        out["hist/f1_%d" % sf] = np.asarray(meta["f1score_histories"][0.0][sf], dtype=np.float64)
    m.eval()
    with torch.no_grad():
        gcs = m.GC(cfg["gc_mode"], X=val[0][0][:, :max(cfg["L"], cfg["F"]), :], threshold=False, ignore_lag=False,
                   combine_wavelet_representations=True)
    out["final_gc"] = np.stack([np.stack([_np(g) for g in row]) for row in gcs])
    out["f1"] = np.asarray([[REF.metrics.get_f1_score(_np(g).sum(axis=2) / np.max(_np(g).sum(axis=2)),
                                                       true_gc[k].sum(axis=2)) for k, g in enumerate(row)]
                            for row in gcs], dtype=np.float64)
    meta_cfg = dict(cfg)
    meta_cfg["coeff"] = coeff
    meta_cfg["max_iter"] = max_iter
    out["meta"] = np.asarray(json.dumps(meta_cfg))
    np.savez_compressed(os.path.join(HERE, "fit_trace.npz"), **out)
    print("wrote fit_trace")


METRIC_CASES = {
    # (S samples, K estimates, G true graphs, nsup histories, p, L lags of the estimates, true lags)
    "a": dict(S=3, K=3, G=3, nsup=3, p=5, L=2, lags=2, seed=31, ties=False, edge=False),
    "b": dict(S=4, K=4, G=4, nsup=4, p=10, L=4, lags=2, seed=32, ties=True, edge=False),
    "c": dict(S=2, K=3, G=3, nsup=2, p=12, L=9, lags=3, seed=33, ties=False, edge=False),
    "d": dict(S=2, K=2, G=2, nsup=2, p=6, L=3, lags=2, seed=34, ties=True, edge=True),
}


def run_metrics():
    """The reference's per-epoch GC-progress trackers (general_utils/model_utils.py:18-209) on
    seeded estimates: one tracking call each, histories stored per case."""
    mu = REF.model_utils
    out = {}
    for name, c in METRIC_CASES.items():
        rng = np.random.RandomState(c["seed"])
        S, K, G, nsup, p, L = c["S"], c["K"], c["G"], c["nsup"], c["p"], c["L"]
        est = (rng.rand(S, K, p, p, L) - 0.15).astype(np.float32)
        if c["ties"]:
            est = (np.round(est * 4.) / 4.).astype(np.float32)
        gc = (rng.rand(G, p, p, c["lags"]) > 0.6).astype(np.float64)
        if c["edge"]:
            gc[0] = 0.                                  # unknown truth: roc 0.5, no normalisation
            est[0, 1] = -np.abs(est[0, 1]) - 0.1         # all-negative estimate (max < 0)
            est[1, 0, :, :, 0] = 0.                      # exact zeros
        nolag = (rng.rand(S + 3, K, p, p, 1) - 0.2).astype(np.float32)
        cur = [[torch.from_numpy(est[s, k].copy()) for k in range(K)] for s in range(S)]
        GC = [gc[g] for g in range(G)]
        f1, roc = {0.0: [[] for _ in range(nsup)]}, {0.0: [[] for _ in range(nsup)]}
        f1o, roco = {0.0: [[] for _ in range(nsup)]}, {0.0: [[] for _ in range(nsup)]}
        mu.track_receiver_operating_characteristic_stats_for_redcliff_models(GC, cur, f1, roc, remove_self_connections=False)
        mu.track_receiver_operating_characteristic_stats_for_redcliff_models(GC, cur, f1o, roco, remove_self_connections=True)
        dc, dcdd, daff = [[] for _ in range(nsup)], [[] for _ in range(nsup)], [[] for _ in range(nsup)]
        plm = {pl: [[] for _ in range(nsup)] for pl in range(1, p)}
        mu.track_deltacon0_related_stats_for_redcliff_models(GC, cur, p, dc, dcdd, daff, plm, deltaConEps=0.1,
                                                             in_degree_coeff=1., out_degree_coeff=0.5)
        l1 = [[] for _ in range(nsup)]
        mu.track_l1_norm_stats_of_gc_ests_from_redcliff_models([[e.numpy() for e in row] for row in cur], l1)
        cos = {"%dand%d" % (i, j): [] for i in range(K) for j in range(K) if i < j}
        mu.track_cosine_similarity_stats_of_gc_ests_from_redcliff_models(
            [[nolag[s, k] for k in range(K)] for s in range(S + 3)], cos, label_offset=0)
        pre = "%s/" % name
        out[pre + "est"] = est
        out[pre + "gc"] = gc
        out[pre + "nolag"] = nolag
        out[pre + "meta"] = np.asarray(json.dumps(c))
        out[pre + "f1"] = np.asarray([h[0] for h in f1[0.0]], dtype=np.float64)
        out[pre + "roc"] = np.asarray([h[0] for h in roc[0.0]], dtype=np.float64)
        out[pre + "f1_off"] = np.asarray([h[0] for h in f1o[0.0]], dtype=np.float64)
        out[pre + "roc_off"] = np.asarray([h[0] for h in roco[0.0]], dtype=np.float64)
        out[pre + "dc"] = np.asarray([h[0] for h in dc], dtype=np.float64)
        out[pre + "dcdd"] = np.asarray([h[0] for h in dcdd], dtype=np.float64)
        out[pre + "daff"] = np.asarray([h[0] for h in daff], dtype=np.float64)
        out[pre + "plm"] = np.asarray([[plm[pl][i][0] if plm[pl][i] else np.nan for i in range(nsup)]
                                       for pl in range(1, p)], dtype=np.float64)
        out[pre + "l1"] = np.asarray([float(h[0]) for h in l1], dtype=np.float64)
        out[pre + "cos"] = np.asarray([float(cos[k][0]) for k in sorted(cos)], dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "gc_metrics.npz"), **out)
    print("wrote gc_metrics")


BASE = dict(seed=0, emb="DGCNN", p=6, L=3, K=3, nsup=3, h=8, F=5, n=3, H=7, eh=0, S=1, sigmoid=False,
            smoothing_class=True, gc_mode="conditional_factor_fixed_embedder",
            fwd_mode="apply_factor_weights_after_sim_completion",
            training_mode="pretrain_embedder_then_acclimate_factors_then_combined", pre=1, acc=1,
            epochs=[0, 1, 2, 2], N=32, T=12, label_T=12, data_seed=1, B=16, lrA=5e-3, lrB=5e-3)

SCENARIOS = {
    # published configuration, C1-shaped (DGCNN, K = nsup, Y labelled per time step)
    "dgcnn_c1": dict(BASE),
    # D4IC-shaped: labels (N, K, 1), 2 graph layers, partial last batch
    "dgcnn_d4ic": dict(BASE, p=5, L=2, K=4, nsup=4, h=6, F=4, n=2, H=3, N=40, T=5, label_T=1, data_seed=2, B=16,
                       seed=1),
    # fewer supervised factors than factors, sigmoid restriction, 2-D labels
    "dgcnn_partial_sigmoid": dict(BASE, K=4, nsup=2, sigmoid=True, label_T=0, data_seed=3, seed=2),
    # no supervised factors at all
    "dgcnn_unsup": dict(BASE, K=2, nsup=0, data_seed=4, seed=3),
    # base class (no smoothing penalty)
    "dgcnn_base": dict(BASE, smoothing_class=False, data_seed=5, seed=4),
    # two simulation steps with the smoothing penalty switched on
    "dgcnn_sims2": dict(BASE, S=2, smooth=25.0, T=12, data_seed=6, seed=5),
    # per-step factor weights forward mode
    "dgcnn_eachstep": dict(BASE, S=2, fwd_mode="apply_factor_weights_at_each_sim_step", data_seed=7, seed=6),
    # F == L boundary
    "dgcnn_feql": dict(BASE, L=4, F=4, data_seed=8, seed=7),
    # cEmbedder (fully pinned: no third-party arithmetic)
    "cemb": dict(BASE, emb="cEmbedder", F=4, eh=5, nsup=2, data_seed=9, seed=8),
    # Vanilla embedder (multiple objectives)
    "vanilla": dict(BASE, emb="Vanilla_Embedder", F=5, eh=6, nsup=2, gc_mode="conditional_factor_exclusive",
                    data_seed=10, seed=9),
    # wavelet-decomposed inputs (wavelet_level = 3: 4 series per channel, the only supported
    # count), DGCNN over p * 4 nodes and the cEmbedder with its ranking mask
    "dgcnn_wavelet": dict(BASE, wl=3, p=2, data_seed=11, seed=10),
    "cemb_wavelet": dict(BASE, emb="cEmbedder", wl=3, p=2, F=4, eh=5, nsup=2, data_seed=12, seed=11),
    # the synthetic grid's extreme classes (train/REDCLIFF_S_CMLP_synSysInnovGauss1030_BSCgsSmooth3Parsim.py:
    # numF1_numN3 and numF10_numN6; K = nsup = numF): one factor (no cosine-similarity pairs, the
    # penalty's sum over an empty set) on a 3-channel system, and ten factors on six channels
    "dgcnn_k1p3": dict(BASE, p=3, K=1, nsup=1, data_seed=13, seed=12),
    "dgcnn_k10p6": dict(BASE, K=10, nsup=10, data_seed=14, seed=13),
}

if __name__ == "__main__":
    only = sys.argv[1:]
    for name, cfg in SCENARIOS.items():
        if not only or name in only:
            run_scenario(name, cfg)
    if not only or "cmlp_prox" in only:
        run_prox()
    if not only or "fit_trace" in only:
        run_fit()
    if not only or "gc_metrics" in only:
        run_metrics()
