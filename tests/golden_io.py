"""Helpers to read the golden fixtures written by tests/golden/make_golden.py."""
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SCENARIOS = ["dgcnn_c1", "dgcnn_d4ic", "dgcnn_partial_sigmoid", "dgcnn_unsup", "dgcnn_base", "dgcnn_sims2",
             "dgcnn_eachstep", "dgcnn_feql", "cemb", "vanilla", "dgcnn_k1p3", "dgcnn_k10p6"]


def load(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(d["meta"])) if "meta" in d.files else None
    return d, meta


def state(d, prefix):
    pre = prefix + "/"
    return dict((k[len(pre):], d[k]) for k in d.files if k.startswith(pre))


def embedder_args(meta):
    if meta["emb"] == "DGCNN":
        return [("num_features_per_node", meta["F"]), ("num_graph_conv_layers", meta["n"]),
                ("num_hidden_nodes", meta["H"]), ("sigmoid_eccentricity_coeff", 10.0)]
    if meta["emb"] == "cEmbedder":
        return [("sigmoid_eccentricity_coeff", 10.0), ("lag", meta["F"]), ("hidden", [meta["eh"]])]
    return []


def ctor_args(meta):
    """Positional + keyword arguments of the reference constructor for a fixture."""
    args = (meta["p"], meta["L"], [meta["h"]], meta["F"], [meta.get("eh", 0)], meta["L"], 1, meta["K"], meta["nsup"],
            meta["coeff"], meta["sigmoid"], meta["emb"], embedder_args(meta), meta["gc_mode"], meta["fwd_mode"])
    kw = dict(num_sims=meta["S"], wavelet_level=meta.get("wl"), save_path=None, training_mode=meta["training_mode"],
              num_pretrain_epochs=meta["pre"], num_acclimation_epochs=meta["acc"])
    return args, kw


def batches(d, meta):
    X, Y = d["X"], d["Y"]
    B = meta["B"]
    return [(torch.from_numpy(X[i:i + B]), torch.from_numpy(Y[i:i + B])) for i in range(0, X.shape[0], B)]


def assert_close(name, got, want, rtol=1e-4, atol=1e-5, outliers=0):
    """|got - want| <= atol + rtol*|want| elementwise.  `outliers` elements may exceed that
    bound, but never 10x it (used only where fp32 re-association can flip isolated
    relu/sign near-ties, see tests/test_gpu_parity.py::OUTLIERS)."""
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    assert got.shape == want.shape, "%s: shape %s vs %s" % (name, got.shape, want.shape)
    if want.size == 0:
        return
    nan_g, nan_w = np.isnan(got), np.isnan(want)
    assert np.array_equal(nan_g, nan_w), "%s: NaN pattern differs (%d got, %d want, %d disagree)" % (
        name, int(nan_g.sum()), int(nan_w.sum()), int((nan_g != nan_w).sum()))
    got, want = np.where(nan_w, 0.0, got), np.where(nan_w, 0.0, want)
    err = np.abs(got - want)
    tol = atol + rtol * np.abs(want)
    bad = err > tol
    if outliers and int(bad.sum()) <= outliers:
        bad = err > 10.0 * tol
    assert not bad.any(), "%s: %d/%d mismatches, max abs err %.3e (at want=%.6g)" % (
        name, int(bad.sum()), want.size, float(err.max()), float(want.flat[int(np.argmax(err))]))
