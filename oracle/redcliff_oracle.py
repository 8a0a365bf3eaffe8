"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the REDCLIFF-S cMLP fitting hot path.

This is the checker for the MI355X build.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it; the product package never does.

What it restates (all citations relative to the reference tree):
* ``models/cmlp.py:12-40``            MLP (lag-L Conv1d -> ReLU -> 1x1 Conv1d)
* ``models/cmlp.py:44-101``           cMLP (one MLP per channel)
* ``models/cmlp.py:117-144``          proximal GL / GSGL / H steps
* ``models/cmlp.py:147-203``          cMLP.GC group norms
* ``models/redcliff_factor_score_embedders.py:51-179``  Vanilla embedders
* ``models/redcliff_factor_score_embedders.py:183-331`` cEmbedder
* ``models/redcliff_factor_score_embedders.py:335-392`` + ``models/dgcnn.py:15-64`` DGCNN embedder
* ``models/redcliff_s_cmlp_withStateSmoothing.py:19-146``  constructor (RNG order: embedder, then factors)
* ``...withStateSmoothing.py:253-412``  both forward modes
* ``...withStateSmoothing.py:415-620``  the nine GC modes
* ``...withStateSmoothing.py:624-731``  compute_loss (base class: ``models/redcliff_s_cmlp.py:620-686``)
* ``...withStateSmoothing.py:734-933``  batch_update phase schedule
* ``...withStateSmoothing.py:1650-1790`` validate_training
* ``general_utils/metrics.py:342-381`` cosine-similarity penalty (detached, I subtracted)

The op structure deliberately keeps the reference's per-sample / per-factor Python loops,
autograd and ``torch.optim.Adam``, so its wall time is representative of the reference
CPU path (used as ``cpu_baseline`` kind "port" in bench.py).

Pinning: tests/test_oracle_golden.py checks this file against golden vectors produced
by the reference itself in this container (tests/golden/make_golden.py).  DGCNN
arithmetic comes from oracle/torcheeg_dgcnn.py: "parity unpinned at the torcheeg 1.1.3
boundary".
"""
import math

import numpy as np
import torch
import torch.nn as nn

from oracle.torcheeg_dgcnn import DGCNN as _TorchEEGDGCNN

TRAINING_MODES = (
    "pretrain_embedder_then_acclimate_factors_then_combined",
    "pretrain_embedder_then_post_train_factor_withComboCosSimL1FreezeByEpoch",
    "pretrain_embedder_then_post_train_factor_withComboCosSimL1FreezeByBatch",
    "pretrain_embedder_then_post_train_factor_withL1FreezeByEpoch",
    "pretrain_embedder_then_post_train_factor_withL1FreezeByBatch",
    "pretrain_embedder_then_post_train_factor",
    "pretrain_embedder_and_pretrain_factor_then_combined",
    "pretrain_embedder_then_combined",
    "pretrain_factor_then_combined",
    "combined",
)
GC_MODES = (
    "fixed_factor_exclusive", "raw_embedder", "conditional_factor_exclusive",
    "fixed_embedder_exclusive", "conditional_embedder_exclusive",
    "fixed_factor_fixed_embedder", "conditional_factor_fixed_embedder",
    "fixed_factor_conditional_embedder", "conditional_factor_conditional_embedder",
)


# --------------------------------------------------------------------------- modules
class OMLP(nn.Module):
    """models/cmlp.py:12-35 -- same parameter tree ``layers.{i}.{weight,bias}``."""

    def __init__(self, n_in, lag, hidden):
        super().__init__()
        widths = list(hidden) + [1]
        first = nn.Conv1d(n_in, widths[0], lag)
        nn.init.xavier_uniform_(first.weight)
        mods = [first] + [nn.Conv1d(a, b, 1) for a, b in zip(widths[:-1], widths[1:])]
        self.layers = nn.ModuleList(mods)
        self.lag = lag

    def forward(self, X):
        z = X.transpose(2, 1)
        for i, layer in enumerate(self.layers):
            z = layer(z if i == 0 else torch.relu(z))
        return z.transpose(2, 1)


def _group_norm_stack(weights, ignore_lag):
    dims = (0, 2) if ignore_lag else 0
    return torch.stack([torch.norm(W, dim=dims) for W in weights])


class OCMLP(nn.Module):
    """models/cmlp.py:44-203 (wavelet_level=None path)."""

    def __init__(self, p, lag, hidden):
        super().__init__()
        self.num_chans = p
        self.num_series = p
        self.lag = lag
        self.wavelet_level = None
        self.networks = nn.ModuleList([OMLP(p, lag, hidden) for _ in range(p)])

    def forward(self, X):
        return torch.cat([net(X) for net in self.networks], dim=2)

    def GC(self, threshold=True, ignore_lag=True):
        G = _group_norm_stack([net.layers[0].weight for net in self.networks], ignore_lag)
        return (G > 0).int() if threshold else G

    def prox(self, lam, lr, penalty):
        """models/cmlp.py:117-144"""
        t = lr * lam
        for net in self.networks:
            W = net.layers[0].weight
            lag = W.shape[2]
            if penalty == "GL":
                nrm = torch.norm(W, dim=(0, 2), keepdim=True)
                W.data = (W / torch.clamp(nrm, min=t)) * torch.clamp(nrm - t, min=0.0)
            elif penalty == "GSGL":
                nrm = torch.norm(W, dim=0, keepdim=True)
                W.data = (W / torch.clamp(nrm, min=t)) * torch.clamp(nrm - t, min=0.0)
                nrm = torch.norm(W, dim=(0, 2), keepdim=True)
                W.data = (W / torch.clamp(nrm, min=t)) * torch.clamp(nrm - t, min=0.0)
            elif penalty == "H":
                for i in range(lag):
                    nrm = torch.norm(W[:, :, :i + 1], dim=(0, 2), keepdim=True)
                    W.data[:, :, :i + 1] = (W.data[:, :, :i + 1] / torch.clamp(nrm, min=t)) * torch.clamp(nrm - t, min=0.0)
            else:
                raise ValueError("unsupported penalty: %s" % penalty)


class _DGCNNHolder(nn.Module):
    """models/dgcnn.py:15-64: keeps the ``dgcnn.dgcnn.*`` key path."""

    def __init__(self, p, F, n, H, K):
        super().__init__()
        self.num_channels = p
        self.num_wavelets_per_chan = 1
        self.dgcnn = _TorchEEGDGCNN(F, p, n, H, K)

    def GC(self, threshold=True, combine=False):
        G = self.dgcnn.A
        if combine:  # 1x1 Frobenius blocks == abs (models/dgcnn.py:49-56)
            G = torch.abs(G)
        G = G.T
        return (G > 0).int() if threshold else G


class ODGCNNEmbedder(nn.Module):
    """models/redcliff_factor_score_embedders.py:335-392"""

    def __init__(self, p, F, n, H, ecc, use_sigmoid, K, n_cls):
        super().__init__()
        self.dgcnn = _DGCNNHolder(p, F, n, H, K)
        self.num_features_per_node = F
        self.num_classes = n_cls
        self.use_sigmoid = use_sigmoid
        self.ecc = ecc

    def forward(self, X, use_final_activation=True):
        if X.size(2) != self.num_features_per_node:
            X = torch.transpose(X, 1, 2)
        w = self.dgcnn.dgcnn(X)
        logits = None
        if self.num_classes > 0:
            logits = w[:, :self.num_classes]
            if use_final_activation and self.use_sigmoid:
                logits = torch.sigmoid(logits)
        if self.use_sigmoid:
            w = torch.sigmoid(self.ecc * w)
        return w, logits

    def GC(self, threshold=True, combine_node_feature_edges=False):
        return self.dgcnn.GC(threshold, combine_node_feature_edges)


class OCEmbedder(nn.Module):
    """models/redcliff_factor_score_embedders.py:183-331 (wavelet_level=None)."""

    def __init__(self, p, n_cls, K, use_sigmoid, ecc, lag, hidden):
        super().__init__()
        self.num_class_preds = n_cls
        self.num_factor_preds = K
        self.use_sigmoid = use_sigmoid
        self.ecc = ecc
        self.networks = nn.ModuleList([OMLP(p, lag, hidden) for _ in range(K)])

    def forward(self, X, use_final_activation=True):
        B = X.size(0)
        w = torch.cat([net(X) for net in self.networks], dim=2).view(B, self.num_factor_preds)
        logits = None
        if self.num_class_preds > 0:
            logits = w[:, :self.num_class_preds]
            if use_final_activation and self.use_sigmoid:
                logits = torch.sigmoid(logits)
        if self.use_sigmoid:
            w = torch.sigmoid(self.ecc * w)
        return w, logits

    def GC(self, threshold=True, ignore_lag=True):
        G = _group_norm_stack([net.layers[0].weight for net in self.networks], ignore_lag)
        return (G > 0).int() if threshold else G


class OVanillaEmbedder(nn.Module):
    """models/redcliff_factor_score_embedders.py:51-179 (single / multiple objective)."""

    def __init__(self, p, T_in, K, n_cls, hidden, use_sigmoid, ecc=10.0):
        super().__init__()
        assert len(hidden) == 1
        self.p, self.T_in, self.K, self.n_cls = p, T_in, K, n_cls
        self.use_sigmoid, self.ecc = use_sigmoid, ecc
        kw = T_in - ((T_in - 1) % 2)
        self.series_embedding_layers = nn.Sequential(
            nn.Conv2d(1, hidden[0], (p, kw), stride=1, padding=(0, kw // 2), bias=False), nn.ReLU(),
            nn.Conv2d(hidden[0], hidden[0], (1, T_in), stride=1, padding=0, bias=False), nn.ReLU())
        if n_cls > 0:
            self.unsup_factor_weighting_layer = (
                nn.Linear(hidden[0] - n_cls, K - n_cls, bias=False) if K - n_cls > 0 else None)
        else:
            self.unsup_factor_weighting_layer = nn.Linear(hidden[0], K, bias=False)

    def forward(self, X, use_final_activation=True):
        B = X.size(0)
        e = self.series_embedding_layers(torch.transpose(X, 1, 2).reshape(B, 1, self.p, self.T_in)).view(B, -1)
        if self.n_cls > 0:
            sup = e[:, :self.n_cls]
            if self.unsup_factor_weighting_layer is not None:
                w = torch.cat((sup, self.unsup_factor_weighting_layer(e[:, self.n_cls:]).view(B, self.K - self.n_cls)), 1)
            else:
                w = sup
            w = w.view(B, self.K)
            if self.use_sigmoid:
                w = torch.sigmoid(self.ecc * w)
            logits = e[:, :self.n_cls]
            if use_final_activation and self.use_sigmoid:
                logits = torch.sigmoid(logits)
            return w, logits
        w = self.unsup_factor_weighting_layer(e).view(B, self.K)
        if self.use_sigmoid:
            w = torch.sigmoid(self.ecc * w)
        return w, None


# --------------------------------------------------------------------------- model
class OracleREDCLIFF(nn.Module):
    """Restatement of REDCLIFF_S_CMLP_withStateSmoothing (with_smoothing=True) and of the
    base REDCLIFF_S_CMLP (with_smoothing=False).  Same constructor signature as
    ``models/redcliff_s_cmlp_withStateSmoothing.py:19-23``."""

    def __init__(self, num_chans, gen_lag, gen_hidden, embed_lag, embed_hidden_sizes, num_in_timesteps,
                 num_out_timesteps, num_factors, num_supervised_factors, coeff_dict, use_sigmoid_restriction,
                 factor_score_embedder_type, factor_score_embedder_args, primary_gc_est_mode, forward_pass_mode,
                 num_sims=1, wavelet_level=None, save_path=None,
                 training_mode="pretrain_embedder_and_pretrain_factor_then_combined", num_pretrain_epochs=0,
                 num_acclimation_epochs=0, STATE_SCORE_SMOOTHING_EPSILON=0.0001, with_smoothing=True):
        super().__init__()
        assert wavelet_level is None, "oracle covers the wavelet_level=None path only"
        assert training_mode in TRAINING_MODES
        assert forward_pass_mode in ("apply_factor_weights_at_each_sim_step", "apply_factor_weights_after_sim_completion")
        assert primary_gc_est_mode in GC_MODES
        assert factor_score_embedder_type in ("cEmbedder", "DGCNN", "Vanilla_Embedder")
        self.with_smoothing = with_smoothing
        self.num_chans = self.num_series = num_chans
        self.gen_lag, self.embed_lag = gen_lag, embed_lag
        self.gen_hidden = gen_hidden
        self.num_factors_nK = num_factors
        self.num_supervised_factors = num_supervised_factors
        self.num_sims = num_sims
        self.eps_smooth = STATE_SCORE_SMOOTHING_EPSILON
        self.c = dict(coeff_dict)
        self.c.setdefault("FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF", 0.0)
        self.training_mode = training_mode
        self.num_pretrain_epochs = num_pretrain_epochs
        self.num_acclimation_epochs = num_acclimation_epochs
        self.forward_pass_mode = forward_pass_mode
        self.primary_gc_est_mode = primary_gc_est_mode
        self.factor_score_embedder_type = factor_score_embedder_type
        args = [a[1] for a in factor_score_embedder_args]
        if factor_score_embedder_type == "cEmbedder":
            ecc, lag, hidden = args
            self.factor_score_embedder = OCEmbedder(num_chans, num_supervised_factors, num_factors,
                                                    use_sigmoid_restriction, ecc, lag, hidden)
        elif factor_score_embedder_type == "DGCNN":
            assert primary_gc_est_mode != "conditional_embedder_exclusive"
            F, n, H, ecc = args
            self.factor_score_embedder = ODGCNNEmbedder(num_chans, F, n, H, ecc, use_sigmoid_restriction,
                                                        num_factors, num_supervised_factors)
        else:
            self.factor_score_embedder = OVanillaEmbedder(num_chans, embed_lag, num_factors, num_supervised_factors,
                                                          embed_hidden_sizes, use_sigmoid_restriction)
        self.factors = nn.ModuleList([OCMLP(num_chans, gen_lag, gen_hidden) for _ in range(num_factors)])
        self.gen_model = nn.ModuleList([self.factor_score_embedder, self.factors])

    # ------------------------------------------------------------------ helpers
    @property
    def Lmax(self):
        return max(self.gen_lag, self.embed_lag)

    def _embed(self, X):
        """Embedder on the last embed_lag steps (...withStateSmoothing.py:335-343, :483-486)."""
        win = X[:, -self.embed_lag:, :]
        if self.factor_score_embedder_type == "DGCNN":
            win = torch.transpose(win, 1, 2)
        return self.factor_score_embedder(win)

    # ------------------------------------------------------------------ forward
    def forward(self, X, factor_weightings=None):
        if self.forward_pass_mode == "apply_factor_weights_after_sim_completion":
            return self._forward_after(X, factor_weightings)
        return self._forward_each_step(X, factor_weightings)

    def _forward_after(self, X, fw):
        """...withStateSmoothing.py:326-385"""
        if fw is None:
            fw, logits = self._embed(X)
        else:
            _, logits = self._embed(X)
        if logits is None:
            logits = fw
        labels = [logits for _ in range(self.num_sims)]
        per_factor = []
        for factor in self.factors:
            cur = X[:, -self.gen_lag:, :] + 0.0
            outs = []
            for s in range(self.num_sims):
                if s > 0:
                    prev = outs[-1]
                    cur = prev if prev.size() == cur.size() else torch.cat([cur[:, prev.size(1):, :], prev], dim=1)
                outs.append(factor(cur))
            per_factor.append(torch.cat(outs, dim=1))
        x_sim = None
        for k in range(self.num_factors_nK):
            term = fw[:, k].view(-1, 1, 1) * per_factor[k]
            x_sim = term if x_sim is None else x_sim + term
        return x_sim, per_factor, [fw], labels

    def _forward_each_step(self, X, fw_given):
        """...withStateSmoothing.py:253-323"""
        inputs = [X + 0.0]
        sims, preds_over, fws, labels = [], [], [], []
        for s in range(self.num_sims):
            if s > 0:
                last = sims[-1]
                inputs.append(last if last.size() == inputs[-1].size()
                              else torch.cat([inputs[-1][:, last.size(1):, :], last], dim=1))
            if fw_given is None:
                fw, logits = self._embed(inputs[s])
            else:
                fw = fw_given
                _, logits = self._embed(inputs[s])
            labels.append(fw if logits is None else logits)
            combined, fpreds = None, []
            for k, factor in enumerate(self.factors):
                pred = factor(inputs[s][:, -self.gen_lag:, :])
                term = fw[:, k].view(-1, 1, 1) * pred
                combined = term if combined is None else combined + term
                fpreds.append(pred)
            preds_over.append(fpreds)
            fws.append(fw)
            sims.append(combined)
        return torch.cat(sims, dim=1), preds_over, fws, labels

    # ------------------------------------------------------------------ GC
    def _factor_gcs(self, threshold, ignore_lag):
        ests = [f.GC(threshold=threshold, ignore_lag=ignore_lag) for f in self.factors]
        if ests[0].dim() != 3:
            n = ests[0].size(0)
            ests = [e.view(n, n, 1) for e in ests]
        return ests

    def _raw_embedder_gc(self, threshold, ignore_lag, combine):
        emb = self.factor_score_embedder
        if self.factor_score_embedder_type == "cEmbedder":
            G = emb.GC(threshold=threshold, ignore_lag=ignore_lag)
            if G.dim() != 3:
                G = G.view(self.num_factors_nK, G.size(1), 1)
        elif self.factor_score_embedder_type == "DGCNN":
            G = emb.GC(threshold=threshold, combine_node_feature_edges=combine)
            if G.dim() != 3:
                G = G.view(self.num_series, self.num_series, 1)
        else:
            raise ValueError("raw_embedder GC needs a causal embedder")
        return G

    def _fixed_embedder_gc(self, threshold, ignore_lag, combine):
        G = self._raw_embedder_gc(threshold, ignore_lag, combine)
        if self.factor_score_embedder_type == "DGCNN":
            return G
        Gt = G.transpose(0, 2)
        return torch.matmul(Gt, Gt.transpose(1, 2)).transpose(0, 2)

    def GC(self, gc_est_mode, X=None, threshold=True, ignore_lag=True, combine_wavelet_representations=False,
           rank_wavelets=False):
        combine = combine_wavelet_representations
        ls = min(self.gen_lag, self.embed_lag)
        if gc_est_mode == "fixed_factor_exclusive":
            return [self._factor_gcs(threshold, ignore_lag)]
        if gc_est_mode == "raw_embedder":
            return [[self._raw_embedder_gc(threshold, ignore_lag, combine)]]
        if gc_est_mode == "fixed_embedder_exclusive":
            return [[self._fixed_embedder_gc(threshold, ignore_lag, combine)]]
        if gc_est_mode == "conditional_factor_exclusive":
            fw, _ = self._embed(X)
            fg = self._factor_gcs(threshold, ignore_lag)
            return [[fw[b, k] * fg[k] for k in range(fw.size(1))] for b in range(fw.size(0))]
        if gc_est_mode == "conditional_embedder_exclusive":
            if self.factor_score_embedder_type == "DGCNN":
                raise ValueError("conditional_embedder_exclusive is not supported with DGCNN")
            raw = self._raw_embedder_gc(threshold, ignore_lag, combine)
            nv, nl = raw.size(1), raw.size(2)
            fw, _ = self._embed(X)
            out = []
            for b in range(fw.size(0)):
                row = []
                for k in range(fw.size(1)):
                    g = raw[k].view(1, nv, nl).transpose(0, 2)
                    row.append(fw[b, k] * torch.matmul(g, g.transpose(1, 2)).transpose(0, 2))
                out.append(row)
            return out
        if gc_est_mode == "fixed_factor_fixed_embedder":
            fg = self._factor_gcs(threshold, ignore_lag)
            eg = self._fixed_embedder_gc(threshold, ignore_lag, combine)
            if not ignore_lag:
                return [[g[:, :, -ls:] + eg[:, :, -ls:] for g in fg]]
            return [[g + eg for g in fg]]
        if gc_est_mode == "conditional_factor_fixed_embedder":
            cond = self.GC("conditional_factor_exclusive", X, threshold, ignore_lag, combine)
            eg = self._fixed_embedder_gc(threshold, ignore_lag, combine)
            for b in range(X.size(0)):
                for k in range(self.num_factors_nK):
                    cond[b][k] = cond[b][k] + eg if ignore_lag else cond[b][k][:, :, -ls:] + eg[:, :, -ls:]
            return cond
        if gc_est_mode == "fixed_factor_conditional_embedder":
            fg = self._factor_gcs(threshold, ignore_lag)
            cond = self.GC("conditional_embedder_exclusive", X, threshold, ignore_lag, combine)
            for b in range(X.size(0)):
                for k in range(self.num_factors_nK):
                    cond[b][k] = cond[b][k] + fg[k] if ignore_lag else cond[b][k][:, :, -ls:] + fg[k][:, :, -ls:]
            return cond
        if gc_est_mode == "conditional_factor_conditional_embedder":
            a = self.GC("conditional_factor_exclusive", X, threshold, ignore_lag, combine)
            e = self.GC("conditional_embedder_exclusive", X, threshold, ignore_lag, combine)
            return [[(a[b][k] + e[b][k]) if ignore_lag else (a[b][k][:, :, -ls:] + e[b][k][:, :, -ls:])
                     for k in range(self.num_factors_nK)] for b in range(X.size(0))]
        raise ValueError("GC EST MODE == %s IS NOT SUPPORTED" % gc_est_mode)

    # ------------------------------------------------------------------ loss
    @staticmethod
    def _cos_pairs_detached(mats):
        """general_utils/metrics.py:342-381 with include_diag=False."""
        if len(mats) <= 1:
            return None
        vals = []
        for i in range(len(mats)):
            for j in range(i + 1, len(mats)):
                A, B = mats[i], mats[j]
                eye = torch.zeros(A.size())
                for l in range(A.size(2)):
                    eye[:, :, l] += torch.eye(A.size(0))
                a = (A - eye).flatten().view(1, -1)
                b = (B - eye).flatten().view(1, -1)
                vals.append(torch.nn.functional.cosine_similarity(a, b))
        return torch.Tensor([float(v) for v in vals]).view(1, -1)

    def compute_loss(self, conditioning_X, preds, targets, factor_scores, factor_labels, gc_est_mode,
                     node_dag_scale=0.1, embedder_pretrain_loss=False, factor_pretrain_loss=False):
        c = self.c
        gc = self.GC(gc_est_mode, X=conditioning_X, threshold=False, ignore_lag=True)
        gc_lagged = self.GC(gc_est_mode, X=conditioning_X, threshold=False, ignore_lag=False)
        mse = nn.MSELoss(reduction="mean")
        forecast = c["FORECAST_COEFF"] * sum(mse(preds[:, :, i], targets[:, :, i]) for i in range(self.num_series))
        factor = torch.tensor([0.0], requires_grad=True)
        nsup = self.num_supervised_factors
        if factor_scores is not None and factor_scores[0] is not None and nsup > 0:
            Lm = self.Lmax
            if factor_labels.dim() == 3 and factor_labels.size(2) > Lm:
                for y, yhat in zip([factor_labels[:, :, Lm + l] for l in range(factor_labels.size(2) - Lm)], factor_scores):
                    factor = factor + c["FACTOR_SCORE_COEFF"] * mse(yhat[:, :nsup], y[:, :nsup])
            else:
                y = factor_labels[:, :, 0] if factor_labels.dim() == 3 else factor_labels
                yhat = factor_scores[0]
                for extra in factor_scores[1:]:
                    yhat = yhat + extra
                yhat = yhat / (1. * len(factor_scores))
                factor = factor + c["FACTOR_SCORE_COEFF"] * mse(yhat[:, :nsup], y[:, :nsup])
        fw_l1 = c["FACTOR_WEIGHT_L1_COEFF"] * (torch.norm(factor_scores[0], 1) - 1.)
        smooth = torch.tensor([0.0], requires_grad=True)
        if self.with_smoothing:
            if self.num_sims == 2:
                d = factor_scores[0] - factor_scores[1]
                d = d * (d > self.eps_smooth)
                smooth = torch.sum(d ** 2.)
            elif self.num_sims > 2:
                for idx, (s0, s1, s2) in enumerate(zip(factor_scores[:-2], factor_scores[1:-1], factor_scores[2:])):
                    full = s2 - s0
                    d21 = s2 - s1
                    smooth = smooth + torch.sum((d21 * torch.gt(torch.abs(d21), torch.abs(full))) ** 2.)
                    if idx == 0:
                        d10 = s1 - s0
                        smooth = smooth + torch.sum((d10 * torch.gt(torch.abs(d10), torch.abs(full))) ** 2.)
            smooth = smooth * c["FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF"]
        cos_pen, adj = None, None
        for b in range(len(gc)):
            if len(gc[b]) > 1:
                v = c["FACTOR_COS_SIM_COEFF"] * torch.sum(self._cos_pairs_detached(gc[b]))
                cos_pen = v if cos_pen is None else cos_pen + v
            for G in gc_lagged[b]:
                v = c["ADJ_L1_REG_COEFF"] * sum(torch.log(torch.tensor(i + 2.)) * torch.norm(G[:, :, i], 1)
                                               for i in range(G.size(2)))
                adj = v if adj is None else adj + v
        if embedder_pretrain_loss:
            combo = factor + fw_l1 + (smooth if self.with_smoothing else 0.0)
        elif factor_pretrain_loss:
            combo = forecast + fw_l1 + (smooth if self.with_smoothing else 0.0) + adj
            if cos_pen is not None:
                combo = combo + cos_pen
        else:
            combo = forecast + factor + fw_l1 + (smooth if self.with_smoothing else 0.0) + adj
            if cos_pen is not None:
                combo = combo + cos_pen
        terms = [forecast, factor, cos_pen, fw_l1]
        if self.with_smoothing:
            terms.append(smooth)
        terms += [adj, None]
        return combo, terms

    # ------------------------------------------------------------------ training
    def phase(self, epoch_num):
        """...withStateSmoothing.py:741-759"""
        if epoch_num <= self.num_pretrain_epochs - 1:
            return ("pretrain_embedder" if "pretrain_embedder" in self.training_mode else None,
                    "pretrain_factor" if "pretrain_factor" in self.training_mode else None)
        if "acclimate_factors" in self.training_mode and epoch_num <= self.num_pretrain_epochs + self.num_acclimation_epochs - 1:
            return ("acclimate",)
        if "combined" in self.training_mode:
            return ("combined",)
        if "post_train_factor" in self.training_mode:
            return ("post_train",)
        raise NotImplementedError()

    def _step_loss(self, X, Y, output_length, **flags):
        Lm = self.Lmax
        x_sims, _, _, labels = self.forward(X[:, :Lm, :])
        tgt = X[:, Lm:Lm + self.num_sims * output_length, :]
        return self.compute_loss(X[:, :self.embed_lag, :], x_sims, tgt, labels, Y, self.primary_gc_est_mode, **flags)

    def batch_update(self, epoch_num, batch_num, X, Y, optimizerA, optimizerB, output_length):
        """...withStateSmoothing.py:734-933 without the Freeze* bookkeeping."""
        ph = self.phase(epoch_num)
        if "pretrain_embedder" in ph:
            self.factor_score_embedder.train()
            optimizerA.zero_grad()
            loss, _ = self._step_loss(X, Y, output_length, embedder_pretrain_loss=True)
            loss.backward()
            optimizerA.step()
        if "pretrain_factor" in ph or "acclimate" in ph:
            self.factor_score_embedder.eval()
            optimizerB.zero_grad()
            loss, _ = self._step_loss(X, Y, output_length, factor_pretrain_loss=True)
            loss.backward()
            optimizerB.step()
        if "combined" in ph:
            self.factor_score_embedder.train()
            optimizerA.zero_grad()
            optimizerB.zero_grad()
            loss, _ = self._step_loss(X, Y, output_length)
            loss.backward()
            optimizerA.step()
            optimizerB.step()
        if "post_train" in ph:
            self.factor_score_embedder.eval()
            optimizerB.zero_grad()
            loss, _ = self._step_loss(X, Y, output_length, factor_pretrain_loss=True)
            loss.backward()
            optimizerB.step()

    @torch.no_grad()
    def validate(self, batches, output_length=1):
        """...withStateSmoothing.py:1650-1790 -> dict of coefficient-normalised averages."""
        self.factor_score_embedder.eval()
        c = self.c
        keys = ["forecast", "factor", "cos", "fw_l1", "smooth", "adj", "combo"]
        acc = dict((k, 0.0) for k in keys)
        for X, Y in batches:
            combo, t = self._step_loss(X, Y, output_length)
            if not self.with_smoothing:
                t = t[:4] + [torch.tensor([0.0])] + t[4:]
            f, fs, cs, l1, sm, ad = [None if v is None else float(v) for v in t[:6]]
            acc["forecast"] += f / c["FORECAST_COEFF"] if c["FORECAST_COEFF"] > 0 else f
            acc["factor"] += fs / c["FACTOR_SCORE_COEFF"] if c["FACTOR_SCORE_COEFF"] > 0 else fs
            if c["FACTOR_COS_SIM_COEFF"] > 0:
                cs = cs / c["FACTOR_COS_SIM_COEFF"] if cs is not None else 0.0
            acc["cos"] += cs
            acc["fw_l1"] += l1 / c["FACTOR_WEIGHT_L1_COEFF"] if c["FACTOR_WEIGHT_L1_COEFF"] > 0 else l1
            acc["smooth"] += sm / c["FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF"] if c["FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF"] > 0 else sm
            acc["adj"] += ad / c["ADJ_L1_REG_COEFF"] if c["ADJ_L1_REG_COEFF"] > 0 else ad
            acc["combo"] += float(combo)
        n = len(batches)
        return dict((k, v / n) for k, v in acc.items())


def make_optimizers(model, embed_lr, embed_eps, embed_wd, gen_lr, gen_eps, gen_wd):
    """general_utils/model_utils.py:747-762"""
    oA = torch.optim.Adam(model.gen_model[0].parameters(), lr=embed_lr, betas=(0.9, 0.999), eps=embed_eps,
                          weight_decay=embed_wd)
    oB = torch.optim.Adam(model.gen_model[1].parameters(), lr=gen_lr, betas=(0.9, 0.999), eps=gen_eps,
                          weight_decay=gen_wd)
    return oA, oB


def f1_score_graph(A_hat, A):
    """general_utils/metrics.py:396-430"""
    A_hat = torch.as_tensor(np.asarray(A_hat))
    A = torch.as_tensor(np.asarray(A))
    pp, pn = 1. * (A_hat > 0.), 1. * (A_hat == 0.)
    lp, ln = 1. * (A > 0.), 1. * (A == 0.)
    tp, tn = pp * lp, pn * ln
    fp, fn = pp - tp, pn - tn
    prec = torch.sum(tp) / (torch.sum(tp) + torch.sum(fp))
    rec = torch.sum(tp) / (torch.sum(tp) + torch.sum(fn))
    if float(prec + rec) == 0.:
        return 0.
    return float(2. * (prec * rec) / (prec + rec))


def reference_coeffs(K, p, forecast=10.0, factor=100.0, cos=1.0, fw_l1=1e-3, smooth=0.0, adj=0.1):
    """Driver coefficient rescaling (train/REDCLIFF_S_CMLP_synSysInnovGauss1030_BSCgsSmooth3Parsim.py:98-108)."""
    denom = sum(float(i) for i in range(1, K)) if K > 1 else 1.0
    return {
        "FORECAST_COEFF": forecast, "FACTOR_SCORE_COEFF": factor, "FACTOR_COS_SIM_COEFF": cos / denom,
        "FACTOR_WEIGHT_L1_COEFF": fw_l1, "FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF": smooth,
        "ADJ_L1_REG_COEFF": adj * (1. / K) * (1. / math.sqrt(p ** 2. - 1.)),
        "DAGNESS_REG_COEFF": 0.0, "DAGNESS_LAG_COEFF": 0.0, "DAGNESS_NODE_COEFF": 0.0,
    }
