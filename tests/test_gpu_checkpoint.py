"""Checkpoint / resume: the files save_checkpoint writes
(final_best_model.bin, training_meta_data_and_hyper_parameters.pkl; ...withStateSmoothing.py:
936-990) reload in a fresh process to the same GC estimates and state, and
resume_training_from_checkpoint + fit (:209-251, :1229-1277) continues a fit exactly."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from test_gpu_replicas import data, make, opts

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HKEYS = ("avg_forecasting_loss", "avg_factor_loss", "avg_factor_cos_sim_penalty", "avg_fw_l1_penalty",
         "avg_adj_penalty", "avg_combo_loss")

CHILD = r"""
import sys, json
import numpy as np, torch
sys.path.insert(0, %(root)r); sys.path.insert(0, %(pkg)r)
m = torch.load(%(path)r, weights_only=False)   # this package's own pickled module
m = m.cuda().eval()
X = torch.from_numpy(np.load(%(x)r)).cuda()
with torch.no_grad():
    g = m.GC(m.primary_gc_est_mode, X=X, threshold=False, ignore_lag=False, combine_wavelet_representations=True)
    w, _ = m.factor_score_embedder(X[:, -m.embed_lag:, :].transpose(1, 2))
out = {"gc": np.stack([np.stack([t.cpu().numpy() for t in row]) for row in g]), "w": w.cpu().numpy()}
for k, v in m.state_dict().items():
    out["sd/" + k] = v.cpu().numpy()
np.savez(%(out)r, **out)
"""


def test_checkpoint_reloads_in_fresh_process(tmp_path):
    torch.manual_seed(0)
    m = make(0, 10.0, 0.1)
    oA, oB = opts(m, 5e-4, 2e-4)
    train, val = data(64 * 2, seed=3), data(64, seed=4)
    m.fit(str(tmp_path), train, oA, oB, 4, 1, 1, 4, val, lookback=1, check_every=1, verbose=0)
    path = os.path.join(str(tmp_path), "final_best_model.bin")
    for f in ("final_best_model.bin", "training_meta_data_and_hyper_parameters.pkl", "optimizer_state.pt"):
        assert os.path.exists(os.path.join(str(tmp_path), f)), f
    X = val[0][0][:8, :20].numpy()
    np.save(str(tmp_path / "x.npy"), X)
    outp = str(tmp_path / "child.npz")
    code = CHILD % dict(root=ROOT, pkg=os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"),
                        path=path, x=str(tmp_path / "x.npy"), out=outp)
    subprocess.run([sys.executable, "-c", code], check=True, timeout=300)
    got = np.load(outp)
    m.eval()
    Xd = torch.from_numpy(X).cuda()
    with torch.no_grad():
        g = m.GC(m.primary_gc_est_mode, X=Xd, threshold=False, ignore_lag=False, combine_wavelet_representations=True)
        w, _ = m.factor_score_embedder(Xd[:, -m.embed_lag:, :].transpose(1, 2))
    np.testing.assert_array_equal(got["gc"], np.stack([np.stack([t.cpu().numpy() for t in row]) for row in g]))
    np.testing.assert_array_equal(got["w"], w.cpu().numpy())
    for k, v in m.state_dict().items():
        np.testing.assert_array_equal(got["sd/" + k], v.cpu().numpy(), err_msg=k)
    # compact: the file holds one model's parameters, not the engine's or a pack's storage
    nparam = sum(t.numel() for t in m.parameters())
    assert os.path.getsize(path) < 4 * nparam * 1.5 + 2 ** 20


def test_resume_from_checkpoint_continues_exactly(tmp_path):
    """Uninterrupted fit of 7 epochs vs (fit stopped after epoch 2 + resume): the checkpoint of
    epoch 2 (pretrain / acclimation epochs: best_it == it, so final_best_model.bin is the current
    model) plus optimizer_state.pt make the resumed fit identical -- loss histories, best epoch,
    final parameters bit for bit."""
    train, val = data(64 * 2 + 24, seed=3), data(64, seed=4)
    kw = dict(lookback=2, check_every=1, verbose=0)

    def fresh():
        m = make(0, 10.0, 0.1, pre=2, acc=2)
        return m, opts(m, 5e-4, 2e-4)
    full, (fA, fB) = fresh()
    full.fit(None, train, fA, fB, 4, 1, 1, 7, val, **kw)
    part, (pA, pB) = fresh()
    part.fit(str(tmp_path), train, pA, pB, 4, 1, 1, 3, val, **kw)  # epochs 0..2, checkpoint at 2
    res = torch.load(os.path.join(str(tmp_path), "final_best_model.bin"), weights_only=False).cuda()
    res.resume_training_from_checkpoint(os.path.join(str(tmp_path), "training_meta_data_and_hyper_parameters.pkl"),
                                        load_optimizer_state=True)
    assert res.chkpt_best_it == 2
    rA, rB = opts(res, 5e-4, 2e-4)
    res.train()
    res.fit(None, train, rA, rB, 4, 1, 1, 7, val, **kw)
    ha, hb = full.fit_history, res.fit_history
    assert hb["best_it"] == ha["best_it"]
    for k in HKEYS:
        assert hb[k] == ha[k], k
    sa, sb = full.state_dict(), res.state_dict()
    for k in sa:
        np.testing.assert_array_equal(sb[k].cpu().numpy(), sa[k].cpu().numpy(), err_msg=k)
