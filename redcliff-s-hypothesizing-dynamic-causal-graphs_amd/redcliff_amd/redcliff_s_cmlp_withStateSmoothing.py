"""REDCLIFF_S_CMLP_withStateSmoothing on MI355X -- drop-in for
models/redcliff_s_cmlp_withStateSmoothing.py (the class every published run uses).

Same constructor signature, parameter tree (state_dict keys), seeded initialisation,
``forward`` / ``GC`` / ``compute_loss`` / ``batch_update`` / ``validate_training`` /
``fit`` / ``save_checkpoint`` call contracts.  The numerical work of a training step
runs in the fused gfx950 kernel chain of libredcliff_hip.so (redcliff_amd.engine):
the embedder, the K x p factor networks, the conditional-GC penalties, the backward
pass and both Adam updates.  There is no CPU / eager fallback: on a host without the
HIP library or without a GPU the compute methods raise.

Scope of the fused path: DGCNN embedder, one hidden factor
layer, num_sims == 1, factor weights applied after simulation, embed_lag >= gen_lag,
primary GC mode conditional_factor_fixed_embedder -- the published configuration.
Other combinations are accepted by the constructor (checkpoint compatibility) and raise
NotImplementedError when trained.
"""
import math
import weakref

import numpy as np
import torch
import torch.nn as nn

from . import _native as nat
from . import autograd as AG
from . import metrics as M
from .cmlp import cMLP
from .engine import FitEngine, phase_of_epoch, select_labels
from .redcliff_factor_score_embedders import (DGCNN_Embedder, MLPClassifierForMultipleObjectives,
                                              MLPClassifierForSingleObjective, cEmbedder)

TRAINING_MODES = [
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
]
POSSIBLE_GC_EST_MODES = [
    "fixed_factor_exclusive", "raw_embedder", "conditional_factor_exclusive", "fixed_embedder_exclusive",
    "conditional_embedder_exclusive", "fixed_factor_fixed_embedder", "conditional_factor_fixed_embedder",
    "fixed_factor_conditional_embedder", "conditional_factor_conditional_embedder",
]


class REDCLIFF_S_CMLP_withStateSmoothing(nn.Module):
    _WITH_SMOOTHING = True

    def __init__(self, num_chans, gen_lag, gen_hidden, embed_lag, embed_hidden_sizes, num_in_timesteps,
                 num_out_timesteps, num_factors, num_supervised_factors, coeff_dict, use_sigmoid_restriction,
                 factor_score_embedder_type, factor_score_embedder_args, primary_gc_est_mode, forward_pass_mode,
                 num_sims=1, wavelet_level=None, save_path=None,
                 training_mode="pretrain_embedder_and_pretrain_factor_then_combined", num_pretrain_epochs=0,
                 num_acclimation_epochs=0, STATE_SCORE_SMOOTHING_EPSILON=0.0001):
        super().__init__()
        self.MAX_NUM_SAMPS_FOR_GC_VIS = 5
        self.MAX_NUM_SAMPS_FOR_GC_PROGRESS_TRACKING = 40
        self.STATE_SCORE_SMOOTHING_EPSILON = STATE_SCORE_SMOOTHING_EPSILON
        self.num_chans = num_chans
        # wavelet-decomposed inputs: num_chans * (wavelet_level + 1) series (:31-35)
        self.num_series = num_chans if wavelet_level is None else num_chans * (wavelet_level + 1)
        self.gen_lag = gen_lag
        self.gen_hidden = gen_hidden
        self.num_gen_hiddens = len(gen_hidden)
        self.embed_lag = embed_lag
        self.embed_hidden_sizes = embed_hidden_sizes
        self.num_in_timesteps = num_in_timesteps
        self.num_out_timesteps = num_out_timesteps
        self.num_factors_nK = num_factors
        self.num_supervised_factors = num_supervised_factors
        self.coeff_dict = coeff_dict
        self.FORECAST_COEFF = coeff_dict["FORECAST_COEFF"]
        self.FACTOR_SCORE_COEFF = coeff_dict["FACTOR_SCORE_COEFF"]
        self.FACTOR_COS_SIM_COEFF = coeff_dict["FACTOR_COS_SIM_COEFF"]
        self.FACTOR_WEIGHT_L1_COEFF = coeff_dict["FACTOR_WEIGHT_L1_COEFF"]
        if self._WITH_SMOOTHING:
            self.FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF = coeff_dict["FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF"]
        self.ADJ_L1_REG_COEFF = coeff_dict["ADJ_L1_REG_COEFF"]
        self.DAGNESS_REG_COEFF = coeff_dict["DAGNESS_REG_COEFF"]
        self.DAGNESS_LAG_COEFF = coeff_dict["DAGNESS_LAG_COEFF"]
        self.DAGNESS_NODE_COEFF = coeff_dict["DAGNESS_NODE_COEFF"]
        self.num_sims = num_sims
        self.wavelet_level = wavelet_level
        assert training_mode in TRAINING_MODES
        self.training_mode = training_mode
        assert (num_pretrain_epochs > 0) if "pretrain" in training_mode else (num_pretrain_epochs == 0)
        assert (num_acclimation_epochs > 0) if "acclimate" in training_mode else (num_acclimation_epochs == 0)
        self.num_pretrain_epochs = num_pretrain_epochs
        self.num_acclimation_epochs = num_acclimation_epochs
        assert forward_pass_mode in ["apply_factor_weights_at_each_sim_step", "apply_factor_weights_after_sim_completion"]
        self.forward_pass_mode = forward_pass_mode
        self.supervised_loss_fn = nn.MSELoss(reduction="mean")
        self.use_sigmoid_restriction = use_sigmoid_restriction
        assert factor_score_embedder_type in ["cEmbedder", "DGCNN", "Vanilla_Embedder"]
        self.CAUSAL_EMBEDDER_TYPES = ["cEmbedder", "DGCNN"]
        self.factor_score_embedder_type = factor_score_embedder_type
        self.factor_score_embedder_args = factor_score_embedder_args
        self.POSSIBLE_GC_EST_MODES = list(POSSIBLE_GC_EST_MODES)
        assert primary_gc_est_mode in POSSIBLE_GC_EST_MODES
        self.primary_gc_est_mode = primary_gc_est_mode
        args = [a[1] for a in factor_score_embedder_args]
        # construction order (embedder first, then factors) fixes the RNG stream (:111-144)
        if factor_score_embedder_type == "cEmbedder":
            self.factor_score_embedder = cEmbedder(num_chans, num_supervised_factors, num_factors,
                                                   use_sigmoid_restriction, *args, wavelet_level, save_path)
        elif factor_score_embedder_type == "DGCNN":
            assert primary_gc_est_mode != "conditional_embedder_exclusive"
            assert len(factor_score_embedder_args) == 4
            wl = 0 if wavelet_level is None else wavelet_level  # num_wavelets_per_chan (:119-122)
            self.factor_score_embedder = DGCNN_Embedder(num_chans, wl + 1, *args, use_sigmoid_restriction, num_factors,
                                                        num_supervised_factors)
        else:
            if num_supervised_factors > 0:
                self.factor_score_embedder = MLPClassifierForMultipleObjectives(
                    self.num_series, embed_lag, num_factors, num_supervised_factors, embed_hidden_sizes,
                    use_sigmoid_restriction)
            else:
                self.factor_score_embedder = MLPClassifierForSingleObjective(
                    self.num_series, embed_lag, num_factors, embed_hidden_sizes, use_sigmoid_restriction)
        self.factors = nn.ModuleList([cMLP(num_chans, gen_lag, gen_hidden, wavelet_level=wavelet_level,
                                           save_path=save_path) for _ in range(num_factors)])
        self.gen_model = nn.ModuleList([self.factor_score_embedder, self.factors])
        self._engine = None
        if isinstance(self.factor_score_embedder, DGCNN_Embedder):
            self.factor_score_embedder.owner = weakref.ref(self)

    # ------------------------------------------------------------------ plumbing
    def __getstate__(self):
        st = self.__dict__.copy()
        st["_engine"] = None
        st.pop("_generic_path", None)
        return st

    def __setstate__(self, state):
        """torch.load / deepcopy: re-attach the DGCNN embedder to this model, so
        ``model.factor_score_embedder(x)`` (general_utils/misc.py:66,79) works on a loaded model;
        the engine itself is created lazily on the first GPU call."""
        super().__setstate__(state)
        emb = self.__dict__.get("_modules", {}).get("factor_score_embedder")
        if isinstance(emb, DGCNN_Embedder):
            emb.owner = weakref.ref(self)

    @property
    def Lmax(self):
        return max(self.gen_lag, self.embed_lag)

    def fused_supported(self):
        return (self.factor_score_embedder_type == "DGCNN" and self.num_sims == 1 and self.num_gen_hiddens == 1
                and self.forward_pass_mode == "apply_factor_weights_after_sim_completion"
                and self.embed_lag >= self.gen_lag
                and self.primary_gc_est_mode == "conditional_factor_fixed_embedder")

    def check_device_status(self):
        """Raise if a merged-backward hand-off wait on the device timed out since the last check
        (synchronises; fit() and validate_training check on their own, see engine.FitEngine)."""
        if self._engine is not None:
            self._engine.check_device_status("model.check_device_status")

    def engine(self):
        if not self.fused_supported():
            raise NotImplementedError(
                "the gfx950 fused path covers the published REDCLIFF-S configuration (DGCNN embedder, num_sims=1, "
                "gen_hidden of length 1, weights applied after simulation, embed_lag >= gen_lag, "
                "conditional_factor_fixed_embedder); got embedder=%s num_sims=%d mode=%s gc=%s" % (
                    self.factor_score_embedder_type, self.num_sims, self.forward_pass_mode, self.primary_gc_est_mode))
        A = self.factor_score_embedder.dgcnn.dgcnn.A
        if not A.is_cuda:
            raise RuntimeError("REDCLIFF-S on MI355X: move the model to the GPU first (model.cuda()); "
                               "there is no CPU path")
        nat.lib()
        if self._engine is None or self._engine.device != A.device:
            self._engine = FitEngine(self)
        self.factor_score_embedder.owner = weakref.ref(self)
        return self._engine

    def _generic(self):
        """The generic GPU path (redcliff_amd.generic) for configurations outside the fused chain."""
        W = self.factors[0].networks[0].layers[0].weight
        if not W.is_cuda:
            raise RuntimeError("REDCLIFF-S on MI355X: move the model to the GPU first (model.cuda()); "
                               "there is no CPU path")
        nat.lib()
        g = self.__dict__.get("_generic_path")
        if g is None:
            from .generic import GenericPath
            g = GenericPath(self)
            self.__dict__["_generic_path"] = g
        return g

    def _device(self):
        return self.factors[0].networks[0].layers[0].weight.device

    # ------------------------------------------------------------------ forward
    def _labels_from_w(self, w_raw):
        emb = self.factor_score_embedder
        nsup = self.num_supervised_factors
        w = torch.sigmoid(emb.sigmoid_eccentricity_coeff * w_raw) if emb.use_sigmoid_restriction else w_raw
        if nsup > 0:
            logits = w_raw[:, :nsup]
            if emb.use_sigmoid_restriction:
                logits = torch.sigmoid(logits)
        else:
            logits = None
        return w, logits

    def _embed_windows(self, Xw, use_final_activation=True):
        """DGCNN_Embedder.forward on time-major windows Xw (B, F, p)."""
        if not self.fused_supported():
            from .generic import dgcnn_forward
            emb = self.factor_score_embedder
            w = dgcnn_forward(emb.dgcnn.dgcnn, Xw.to(self._device(), torch.float32).transpose(1, 2))
            logits = None
            if self.num_supervised_factors > 0:
                logits = w[:, :self.num_supervised_factors]
                if use_final_activation and emb.use_sigmoid_restriction:
                    logits = torch.sigmoid(logits)
            if emb.use_sigmoid_restriction:
                w = torch.sigmoid(emb.sigmoid_eccentricity_coeff * w)
            return w, logits
        eng = self.engine()
        Xw = Xw.to(eng.device, torch.float32)
        B, F, p = Xw.shape
        pad = self.Lmax - F
        if pad > 0:
            Xw = torch.cat([torch.zeros(B, pad, p, device=Xw.device, dtype=Xw.dtype), Xw], 1)
        train = self.factor_score_embedder.training
        w_raw = AG.embedder_forward(self, Xw.contiguous(), train)
        w, logits = self._labels_from_w(w_raw)
        if logits is not None and not use_final_activation and self.factor_score_embedder.use_sigmoid_restriction:
            logits = w_raw[:, :self.num_supervised_factors]
        return w, logits

    def forward(self, X, factor_weightings=None):
        """X (B, T, p) -> (x_sim (B, S, p), [per-factor predictions], [w], [state labels] * S)
        (...withStateSmoothing.py:326-412).  Uses the last embed_lag / gen_lag steps of X."""
        if not self.fused_supported():
            return self._generic().forward(X.to(self._device(), torch.float32), factor_weightings)
        if factor_weightings is not None:
            raise NotImplementedError("externally supplied factor_weightings are not supported on the fused path")
        eng = self.engine()
        X = X.to(eng.device, torch.float32)
        if X.shape[1] < self.Lmax:
            raise ValueError("forward needs at least max(gen_lag, embed_lag) time steps")
        Xw = X[:, X.shape[1] - self.Lmax:, :].contiguous()
        train = self.factor_score_embedder.training
        xs, y, w_raw = AG.fused_forward(self, Xw, train)  # a graph when gradients are requested
        w, logits = self._labels_from_w(w_raw)
        if logits is None:
            logits = w
        preds = [y[:, k, :].unsqueeze(1) for k in range(self.num_factors_nK)]
        return xs.unsqueeze(1), preds, [w], [logits for _ in range(self.num_sims)]

    # ------------------------------------------------------------------ GC
    def _factor_gcs(self, threshold, ignore_lag, combine=False, rank=False):
        """cMLP.GC of every factor (models/cmlp.py:147-203: norms, wavelet ranking / combination,
        threshold), each viewed as (n, n, 1) when lag-free (:450-454)."""
        eng = self.engine()
        W0s = [net.layers[0].weight for f in self.factors for net in f.networks]
        if AG.grad_needed(W0s) and not threshold:
            G, G0 = AG.group_norms(list(self.factors))  # differentiable (cmlp.py:147-167)
        else:
            G, G0 = eng.gc_norms()
        ests = [self.factors[k].gc_post(G0[k] if ignore_lag else G[k], ignore_lag, combine, rank)
                for k in range(self.num_factors_nK)]
        ests = [e.view(e.size(0), e.size(0), 1) if e.dim() == 2 else e for e in ests]
        return [(e > 0).int() for e in ests] if threshold else ests

    def _embedder_gc(self, threshold, combine):
        G = self.factor_score_embedder.GC(threshold=threshold, combine_node_feature_edges=combine)
        assert G.size(0) == self.num_series  # :472 (a combined wavelet graph fails here, as in the reference)
        return G.view(self.num_series, self.num_series, 1)

    def _conditional_gc_stack(self, gc_est_mode, X, threshold, ignore_lag, comb, rank=False):
        """The conditional GC estimates of every window as one (B, K, p, p, L') tensor: the
        reference's per-(sample, factor) products (:481-498, :565-580) as one broadcast (the
        same element-wise operations, so the same values)."""
        ls = min(self.gen_lag, self.embed_lag)
        w, _ = self.factor_score_embedder(torch.transpose(X[:, -self.embed_lag:, :], 1, 2))
        fg = torch.stack(self._factor_gcs(threshold, ignore_lag, comb, rank))  # (K, p, p, L')
        est = w[:, :, None, None, None] * fg[None]
        if gc_est_mode == "conditional_factor_fixed_embedder":
            eg = self._embedder_gc(threshold, comb)
            est = est + eg if ignore_lag else est[..., -ls:] + eg[:, :, -ls:]
        return est

    def GC(self, gc_est_mode, X=None, threshold=True, ignore_lag=True, combine_wavelet_representations=False,
           rank_wavelets=False):
        """The nine GC estimate modes of ...withStateSmoothing.py:415-620 (DGCNN embedder)."""
        if not self.fused_supported():
            Xd = None if X is None else X.to(self._device(), torch.float32)
            return self._generic().GC(gc_est_mode, Xd, threshold, ignore_lag, combine_wavelet_representations,
                                      rank_wavelets)
        if self.factor_score_embedder_type != "DGCNN":
            raise NotImplementedError("GC on the fused path is implemented for the DGCNN embedder")
        self.engine()  # binds the embedder to this model's kernels (a fresh / loaded model may call GC first)
        ls = min(self.gen_lag, self.embed_lag)
        comb, rank = combine_wavelet_representations, rank_wavelets
        if gc_est_mode == "fixed_factor_exclusive":
            return [self._factor_gcs(threshold, ignore_lag, comb, rank)]
        if gc_est_mode in ("raw_embedder", "fixed_embedder_exclusive"):
            return [[self._embedder_gc(threshold, comb)]]
        if gc_est_mode in ("conditional_embedder_exclusive", "fixed_factor_conditional_embedder",
                           "conditional_factor_conditional_embedder"):
            raise ValueError("conditional_embedder_exclusive is not supported for model with DGCNN factor score "
                             "embedder type")
        if gc_est_mode == "fixed_factor_fixed_embedder":
            fg = self._factor_gcs(threshold, ignore_lag, comb, rank)
            eg = self._embedder_gc(threshold, comb)
            if not ignore_lag:
                return [[g[:, :, -ls:] + eg[:, :, -ls:] for g in fg]]
            return [[g + eg for g in fg]]
        if gc_est_mode in ("conditional_factor_exclusive", "conditional_factor_fixed_embedder"):
            est = self._conditional_gc_stack(gc_est_mode, X, threshold, ignore_lag, comb, rank)
            return [[est[b, k] for k in range(est.size(1))] for b in range(est.size(0))]
        raise ValueError("GC EST MODE == " + str(gc_est_mode) + " IS NOT SUPPORTED")

    # ------------------------------------------------------------------ loss (values)
    def compute_loss(self, conditioning_X, preds, targets, factor_scores, factor_labels, gc_est_mode,
                     node_dag_scale=0.1, embedder_pretrain_loss=False, factor_pretrain_loss=False):
        """Loss terms of ...withStateSmoothing.py:624-731.  A graph tensor whenever gradients are
        enabled (the reference calls .backward() on it, :783): forward, GC and the embedder are
        autograd Functions over the fused kernels (redcliff_amd.autograd); the fused
        batch_update does not use this method (its backward is fused)."""
        if not self.fused_supported():
            dev = self._device()
            return self._generic().compute_loss(conditioning_X.to(dev, torch.float32), preds, targets.to(dev),
                                                factor_scores, factor_labels, gc_est_mode,
                                                embedder_pretrain_loss=embedder_pretrain_loss,
                                                factor_pretrain_loss=factor_pretrain_loss)
        dev = self._device()
        return self._fused_loss_values(conditioning_X.to(dev, torch.float32), preds, targets.to(dev), factor_scores,
                                       factor_labels, gc_est_mode, embedder_pretrain_loss, factor_pretrain_loss)

    def _fused_loss_values(self, conditioning_X, preds, targets, factor_scores, factor_labels, gc_est_mode,
                           embedder_pretrain_loss, factor_pretrain_loss):
        gc = self.GC(gc_est_mode, X=conditioning_X, threshold=False, ignore_lag=True)
        gc_lagged = self.GC(gc_est_mode, X=conditioning_X, threshold=False, ignore_lag=False)
        dev = preds.device
        forecast = self.FORECAST_COEFF * sum(self.supervised_loss_fn(preds[:, :, i], targets[:, :, i])
                                             for i in range(self.num_series))
        factor = torch.zeros(1, device=dev)
        nsup = self.num_supervised_factors
        if factor_scores is not None and factor_scores[0] is not None and nsup > 0:
            lab = select_labels(factor_labels.to(dev), factor_labels.size(1), self.Lmax)
            yhat = sum(factor_scores) / (1. * len(factor_scores)) if not (
                factor_labels.dim() == 3 and factor_labels.size(2) > self.Lmax) else factor_scores[0]
            factor = factor + self.FACTOR_SCORE_COEFF * self.supervised_loss_fn(yhat[:, :nsup], lab[:, :nsup])
        fw_l1 = self.FACTOR_WEIGHT_L1_COEFF * (torch.norm(factor_scores[0], 1) - 1.)
        smooth = torch.zeros(1, device=dev)
        # the per-(sample, factor) loops of :696-715 over stacked estimates: one batched
        # cosine per factor pair (values only: the reference's torch.Tensor(list) drops the
        # gradient, general_utils/metrics.py:380) and one batched lag-weighted L1
        g0 = torch.stack([torch.stack(list(row)) for row in gc])          # (B, K', p, p, 1)
        gl = torch.stack([torch.stack(list(row)) for row in gc_lagged])   # (B, K', p, p, L')
        cos_pen = None
        if g0.shape[1] > 1:
            eye = torch.eye(self.num_series, device=dev).view(1, self.num_series, self.num_series, 1)
            v = (g0.detach() - eye).flatten(2)
            pairs = [(i, j) for i in range(v.shape[1]) for j in range(i + 1, v.shape[1])]
            cs = torch.stack([torch.nn.functional.cosine_similarity(v[:, i], v[:, j], dim=1) for i, j in pairs], 1)
            for row in cs.tolist():
                tot = 0.
                for x in row:
                    tot += x
                val = self.FACTOR_COS_SIM_COEFF * tot
                cos_pen = val if cos_pen is None else cos_pen + val
        logw = torch.tensor([math.log(i + 2.) for i in range(gl.shape[-1])], device=dev, dtype=torch.float32)
        adj = self.ADJ_L1_REG_COEFF * (torch.abs(gl).sum(dim=(2, 3)) * logw).sum()
        cos_t = None if cos_pen is None else torch.tensor(cos_pen, device=dev)
        if embedder_pretrain_loss:
            combo = factor + fw_l1 + smooth
        elif factor_pretrain_loss:
            combo = forecast + fw_l1 + smooth + adj + (cos_t if cos_t is not None else 0.)
        else:
            combo = forecast + factor + fw_l1 + smooth + adj + (cos_t if cos_t is not None else 0.)
        terms = [forecast, factor, cos_t, fw_l1]
        if self._WITH_SMOOTHING:
            terms.append(smooth * getattr(self, "FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF", 0.0))
        return combo, terms + [adj, None]

    # ------------------------------------------------------------------ factor prior / re-ordering
    def _load_prior_factors(self, path, allow_pickle):
        """Factor parameter tensors [K][params in module order] of a prior model file.  Default:
        weights-only loading (torch.load(weights_only=True)), which takes a state_dict of the
        model (or of its factors: keys factors.{k}.networks.{j}.layers.{0,1}.{weight,bias}) and
        executes nothing from the file.  A whole pickled module -- what the reference's fit
        writes and loads (:151) -- is unpickled only with allow_pickle=True (trusted files)."""
        import pickle
        dev = self._device()
        try:
            obj = torch.load(path, map_location=dev, weights_only=True)
        except pickle.UnpicklingError as e:  # disallowed globals; truncated files etc. raise as they are
            if not allow_pickle:
                raise RuntimeError(
                    "prior_factors_path %s is not a weights-only file (a pickled module?): pass "
                    "prior_factors_allow_pickle=True for a trusted file, or save the prior model's state_dict()"
                    % path) from e
            obj = torch.load(path, map_location=dev, weights_only=False)
        if isinstance(obj, dict):
            sd = obj.get("state_dict", obj)
            out = []
            for k, f in enumerate(self.factors):
                ts = []
                for name, _ in f.named_parameters():
                    key = "factors.%d.%s" % (k, name)
                    if key not in sd:
                        raise KeyError("prior state_dict has no %s" % key)
                    ts.append(sd[key])
                out.append(ts)
            return out, None
        return [list(f.parameters()) for f in obj.factors], obj

    def initialize_factors_with_prior(self, prior_factors_path=None, X_train=None, cost_criteria="CosineSimilarity",
                                      unsupervised_start_index=0, max_batches=10, allow_pickle=False):
        """...withStateSmoothing.py:149-206.  fit() calls it at the end of factor pretraining
        ("pretrain_factor" modes, :1318-1326) with X_train: the factors are re-ordered so that
        factor i is the one whose (eval-mode) embedder weighting matches label column i best
        (misc.py:83-91, linear sum assignment on the cosine cost), the unmatched ones after.

        The reference re-orders the module objects, so each factor's Adam state moves with it;
        here the factor slots of the packed parameter buffer and of optimizerB's moments are
        permuted, which is the same state.

        ``prior_factors_path``: the factors are replaced by those of a model saved by fit() /
        save_checkpoint (:151-153, loaded the way the reference loads it: a pickled module, so
        only files this package or the reference wrote).  The reference's ``self.factors =
        prior.factors`` leaves optimizerB (built on gen_model[1]) holding the replaced
        parameters, so the loaded factors are never stepped again; on the fused path their
        values are copied into the factor buffer and optimizerB's updates are dropped from
        every later step (engine.step_flags).  gen_model[1] keeps pointing at the live factors
        here, where the reference's still holds the replaced ones."""
        if prior_factors_path is not None:
            tensors, prior = self._load_prior_factors(prior_factors_path, allow_pickle)
            if not self.fused_supported():
                if prior is not None:
                    self.factors = prior.factors  # the reference's move (:152)
                else:
                    with torch.no_grad():
                        for f_dst, ts in zip(self.factors, tensors):
                            for p_dst, p_src in zip(f_dst.parameters(), ts):
                                p_dst.copy_(p_src.detach().to(p_dst.device, p_dst.dtype))
            else:
                eng = self.engine()
                eng.ensure_bound()
                with torch.no_grad():
                    for f_dst, ts in zip(self.factors, tensors):
                        for p_dst, p_src in zip(f_dst.parameters(), ts):
                            p_dst.copy_(p_src.detach().to(p_dst.device, p_dst.dtype))
                eng.invalidate()
                self.__dict__["_factors_detached"] = True
            del prior, tensors
        if X_train is None:
            return
        if unsupervised_start_index != 0:
            # the reference keeps only factors[start:] (:200-205), which changes num_factors
            raise NotImplementedError("unsupervised_start_index != 0 drops factors in the reference")
        Lm = self.Lmax
        preds, labels = [], []
        with torch.no_grad():
            for batch_num, (X, Y) in enumerate(X_train):
                if batch_num >= max_batches:
                    break
                if Y is not None and Y.dim() > 2:
                    Y = Y[:, :, Lm] if Y.size(2) > Lm else Y[:, :, 0]
                self.factor_score_embedder.eval()
                for f in self.factors:
                    f.eval()
                _, _, fw, _ = self.forward(X[:, :Lm, :].to(self._device(), torch.float32))
                preds.append(fw[0].detach().cpu().numpy())
                labels.append(Y.detach().cpu().numpy())
        preds, labels = np.vstack(preds), np.vstack(labels)
        assert preds.ndim == 2 and labels.ndim == 2
        from .evaluation import sort_unsupervised_estimates
        _, est_inds, gt_inds = sort_unsupervised_estimates(
            [preds[:, i] for i in range(preds.shape[1])], [labels[:, i] for i in range(labels.shape[1])],
            cost_criteria=cost_criteria, unsupervised_start_index=0, return_sorting_inds=True)
        order = [None] * len(est_inds)
        for e, g in zip(est_inds, gt_inds):
            order[g] = int(e)
        if any(o is None for o in order):
            raise ValueError("factor matching left a label column without a factor")
        order += [i for i in range(self.num_factors_nK) if i not in est_inds]
        self._permute_factors(order)

    def _permute_factors(self, order):
        """Factor slot i takes the parameters (and optimizerB state) of factor order[i]."""
        if list(order) == list(range(self.num_factors_nK)):
            return
        if not self.fused_supported():  # the reference's own move: a re-ordered ModuleList (:205)
            self.factors = nn.ModuleList([self.factors[i] for i in order])
            return
        eng = self.engine()
        eng.ensure_bound()
        base = eng.fac
        slots = [[((prm.data_ptr() - base.data_ptr()) // 4, prm.numel()) for prm in f.parameters()]
                 for f in self.factors]
        # detached factors (a prior model's): optimizerB's state belongs to the replaced ones
        moments = eng.opt["B"] is not None and not self.__dict__.get("_factors_detached", False)
        bufs = [eng.fac] + ([eng.opt["B"]["m"], eng.opt["B"]["v"]] if moments else [])
        with torch.no_grad():
            for buf in bufs:
                old = buf.clone()
                for i, src in enumerate(order):
                    for (od, n), (os_, n2) in zip(slots[i], slots[src]):
                        assert n == n2
                        buf[od:od + n].copy_(old[os_:os_ + n])
        eng.invalidate()

    def determine_which_factors_need_updates(self, cached_model, training_status_of_each_factor):
        """...withStateSmoothing.py:1132-1172, the Freeze* training modes' per-factor accept /
        revert decision.  Restated as the reference computes it, including its failure: the
        fixed_factor_exclusive lag-free estimates are (p, p, 1) arrays (:444-455), and
        np.linalg.norm(x, ord=1) of a 3-d array raises ValueError ("Improper number of dimensions
        to norm."), so every Freeze* fit of the reference stops with that error at its first
        decision; this method raises the same error at the same point."""
        from .fit_loop import _as_module
        cached_model = _as_module(cached_model)
        with torch.no_grad():
            cached = [x.detach().cpu().numpy() for x in cached_model.GC(
                "fixed_factor_exclusive", X=None, threshold=False, ignore_lag=True)[0]]
            cur = [x.detach().cpu().numpy() for x in self.GC(
                "fixed_factor_exclusive", X=None, threshold=False, ignore_lag=True)[0]]
        K = self.num_factors_nK
        need = [False] * K
        for f in range(K):
            if not training_status_of_each_factor[f]:
                continue
            c_est = cached[f] / np.max(cached[f])
            n_est = cur[f] / np.max(cur[f])
            if "withComboCosSimL1" in self.training_mode:
                cs_c, cs_n = 0., 0.
                for o in range(K):
                    if o != f:
                        cs_c += M.compute_cosine_similarity(c_est, cached[o] / np.max(cached[o]))
                        cs_n += M.compute_cosine_similarity(n_est, cur[o] / np.max(cur[o]))
                cs_c /= (K - 1.)
                cs_n /= (K - 1.)
                if cs_n * np.linalg.norm(n_est, ord=1) < cs_c * np.linalg.norm(c_est, ord=1):
                    need[f] = True
            elif "withL1" in self.training_mode:
                if np.linalg.norm(n_est, ord=1) < np.linalg.norm(c_est, ord=1):
                    need[f] = True
            else:
                raise NotImplementedError()
        return need

    def resume_training_from_checkpoint(self, training_meta_data_path, load_optimizer_state=False):
        """...withStateSmoothing.py:209-251: histories of a previous run; fit() resumes at best_it+1.

        Default = the reference's behaviour: the optimizers are NOT restored, the resumed fit
        starts from the caller's fresh Adam objects (redcliff_s_cmlp.py:245 warns about exactly
        this), so it reproduces the reference's resumed fit on the same files.
        ``load_optimizer_state=True`` (an extension): the Adam state this package's
        save_checkpoint wrote next to the metadata (optimizer_state.pt) is loaded into fit()'s
        optimizers, which makes an interrupted fit continue bit for bit; a missing file raises."""
        import os
        import pickle
        with open(training_meta_data_path, "rb") as f:
            meta = pickle.load(f)  # a file written by this package's (or the reference's) save_checkpoint
        self.chkpt_epoch = meta["epoch"]
        for k, v in meta.items():
            setattr(self, "chkpt_" + k, v)
        if hasattr(self, "chkpt_optimizer_state"):
            del self.chkpt_optimizer_state
        if load_optimizer_state:
            opt_path = os.path.join(os.path.dirname(os.path.abspath(training_meta_data_path)), "optimizer_state.pt")
            if not os.path.exists(opt_path):
                raise FileNotFoundError("load_optimizer_state=True but %s does not exist" % opt_path)
            self.chkpt_optimizer_state = torch.load(opt_path, map_location=self._device(), weights_only=True)

    # ------------------------------------------------------------------ training step
    def batch_update(self, epoch_num, batch_num, X, Y, optimizerA, optimizerB, output_length, best_model=None,
                     training_status_of_each_factor=None, running_factor_score_confusion_matrix=None):
        """One REDCLIFF-S update on a host or device batch (...withStateSmoothing.py:734-933)."""
        best_model, running_factor_score_confusion_matrix = self._batch_update(
            epoch_num, X, Y, optimizerA, optimizerB, output_length, best_model, running_factor_score_confusion_matrix)
        if "FreezeByBatch" in self.training_mode:  # :910-929
            assert best_model is not None
            assert training_status_of_each_factor is not None
            self.determine_which_factors_need_updates(best_model, training_status_of_each_factor)
            # determine_which_factors_need_updates raises on the reference's (p, p, 1) estimates
            raise AssertionError("unreachable: the reference's Freeze decision cannot complete")
        return best_model, running_factor_score_confusion_matrix

    def _batch_update(self, epoch_num, X, Y, optimizerA, optimizerB, output_length, best_model,
                      running_factor_score_confusion_matrix):
        if output_length != 1:
            raise NotImplementedError("output_length must be 1 (num_sims * output_length target steps)")
        kinds = phase_of_epoch(self, epoch_num)
        if not self.fused_supported():
            dev = self._device()
            n = self.num_supervised_factors
            conf = np.zeros((n, n)) if (running_factor_score_confusion_matrix is not None and n > 0) else None
            self._generic().batch_update(kinds, X.to(dev, torch.float32), Y.to(dev, torch.float32), optimizerA,
                                         optimizerB, output_length, conf)
            self._set_module_modes(kinds[-1] if kinds else None)
            if conf is not None:
                running_factor_score_confusion_matrix += conf
            return best_model, running_factor_score_confusion_matrix
        eng = self.engine()
        Xd, lab, st, d = eng.stage(X, Y)
        if running_factor_score_confusion_matrix is not None:
            eng.conf.zero_()
        eng.run_steps(kinds, Xd, lab, st, d, [0], [Xd.shape[0]], optimizerA, optimizerB)
        self._set_module_modes(kinds[-1] if kinds else None)
        if running_factor_score_confusion_matrix is not None and self.num_supervised_factors > 0:
            n = self.num_supervised_factors
            running_factor_score_confusion_matrix += eng.conf.cpu().numpy().reshape(n, n)
        return best_model, running_factor_score_confusion_matrix

    def _set_module_modes(self, kind):
        if kind in ("pretrain_embedder", "combined"):
            self.factor_score_embedder.train()
        elif kind in ("pretrain_factor", "acclimate", "post_train"):
            self.factor_score_embedder.eval()
            for f in self.factors:
                f.train()

    # ------------------------------------------------------------------ validation
    def validate_training(self, X_val, output_length, num_series, factor_score_val_acc_history=None,
                          factor_score_val_tpr_history=None, factor_score_val_tnr_history=None,
                          factor_score_val_fpr_history=None, factor_score_val_fnr_history=None):
        """...withStateSmoothing.py:1650-1790: coefficient-normalised loss terms averaged over batches."""
        if not self.fused_supported():
            for f in self.factors:
                f.eval()
            avg, conf = self._generic().validate(X_val, output_length)
            acc = [avg[k] for k in ("forecast", "factor", "cos", "fw_l1", "smooth", "adj", "combo")] + [1.0]
            return self._validation_tuple(acc, 1.0, conf, factor_score_val_acc_history,
                                          factor_score_val_tpr_history, factor_score_val_tnr_history,
                                          factor_score_val_fpr_history, factor_score_val_fnr_history)
        self.factor_score_embedder.eval()
        for f in self.factors:
            f.eval()
        return self._validate_fused(X_val, False, factor_score_val_acc_history, factor_score_val_tpr_history,
                                    factor_score_val_tnr_history, factor_score_val_fpr_history,
                                    factor_score_val_fnr_history)

    def _validate_fused(self, X_val, fresh_histories, *hists):
        """validate_training on the fused engine without touching the module flags (fit() sets
        them once); fresh_histories: five new confusion-history lists (fit's call)."""
        eng = self.engine()
        ds = eng.cache_dataset(X_val)
        d = eng.workspace(ds["Bmax"], ds["T"])
        acc, conf = eng.run_values(ds["X"], ds["lab"], d, ds["rows"], ds["sizes"])
        eng.check_device_status("validate_training")
        if fresh_histories:
            hists = [[] for _ in range(5)]
        elif not hists:
            hists = [None] * 5
        return self._validation_tuple(acc, float(ds["len"]), conf, *hists)

    def _validation_tuple(self, acc, nb, conf, acc_h, tpr_h, tnr_h, fpr_h, fnr_h, rates=None):
        vals = [acc[nat_i] / nb for nat_i in range(7)]
        forecast, factor, cos, fwl1, smooth, adj, combo = vals
        out = [forecast, factor, cos, fwl1]
        if self._WITH_SMOOTHING:
            out.append(smooth)
        out += [adj, 0.0, 0.0, 0.0, combo]
        if self.num_supervised_factors > 0:
            TPR, TNR, FPR, FNR, ACC = _confusion_rates(conf) if rates is None else rates
            acc_h.append(ACC)
            tpr_h.append(TPR)
            tnr_h.append(TNR)
            fpr_h.append(FPR)
            fnr_h.append(FNR)
            out += [acc_h, tpr_h, tnr_h, fpr_h, fnr_h]
        return tuple(out)

    # ------------------------------------------------------------------ fit
    def fit(self, save_dir, X_train, optimizerA, optimizerB, input_length, output_length, num_sim_steps, max_iter,
            X_val, lookback=5, check_every=50, verbose=1, GC=None, deltaConEps=0.1, in_degree_coeff=1.,
            out_degree_coeff=1., prior_factors_path=None, cost_criteria="CosineSimilarity",
            unsupervised_start_index=0, max_factor_prior_batches=10, stopping_criteria_forecast_coeff=1.,
            stopping_criteria_factor_coeff=1., stopping_criteria_cosSim_coeff=1., save_plots=False,
            prior_factors_allow_pickle=False):
        """Epoch loop of ...withStateSmoothing.py:1175-1647 with the batches resident on the GPU.
        prior_factors_allow_pickle (extension): see initialize_factors_with_prior."""
        from .fit_loop import run_fit
        return run_fit(self, save_dir, X_train, optimizerA, optimizerB, output_length, max_iter, X_val, lookback,
                       check_every, verbose, GC, deltaConEps, in_degree_coeff, out_degree_coeff,
                       (prior_factors_path, cost_criteria, unsupervised_start_index, max_factor_prior_batches,
                        prior_factors_allow_pickle),
                       stopping_criteria_forecast_coeff, stopping_criteria_factor_coeff,
                       stopping_criteria_cosSim_coeff, save_plots)

    def save_checkpoint(self, save_dir, it, best_model, *histories, **kw):
        """final_best_model.bin + training_meta_data_and_hyper_parameters.pkl (:936-990)."""
        from .fit_loop import save_checkpoint
        return save_checkpoint(self, save_dir, it, best_model, *histories, **kw)


def _confusion_rates(cm):
    cm = np.asarray(cm, dtype=np.float64)
    TP = np.diag(cm)
    FP = cm.sum(axis=0) - TP
    FN = cm.sum(axis=1) - TP
    TN = cm.sum() - (FP + FN + TP)
    with np.errstate(divide="ignore", invalid="ignore"):
        return TP / (TP + FN), TN / (TN + FP), FP / (FP + TN), FN / (TP + FN), (TP + TN) / (TP + FP + FN + TN)
