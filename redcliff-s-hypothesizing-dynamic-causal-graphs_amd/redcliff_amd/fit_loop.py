"""REDCLIFF-S ``fit`` (models/redcliff_s_cmlp_withStateSmoothing.py:1175-1647) on the fused engine.

Per epoch: one ``redcliff_train_steps`` call runs every batch of the (device-resident)
training set; the embedder confusion matrix accumulates on the GPU; GC progress is
tracked on the first validation batch (<= 40 windows, host metrics as in the reference);
validation runs as one more kernel call; early stopping, best-model snapshots,
checkpoints and ``restore_parameters`` follow the reference's rules, including its
parity hazards:
  * stopping is evaluated only after pretrain + acclimation epochs, with an equality test
    ``it - best_it == lookback * check_every``; before that best_model is refreshed every epoch;
  * GC tracking slices the SAMPLE list to num_supervised_factors;
  * restore_parameters restores parameters only (BatchNorm running statistics stay).
The resume typo of the reference (redcliff_s_cmlp.py:1237) is not reproduced.
"""
import copy
import os
import pickle as pkl

import numpy as np
import torch

from . import metrics as M
from .engine import phase_of_epoch

HIST_KEYS = ["avg_forecasting_loss", "avg_factor_loss", "avg_factor_cos_sim_penalty", "avg_fw_l1_penalty",
             "avg_fw_smoothing_penalty", "avg_adj_penalty", "avg_dagness_reg_loss", "avg_dagness_lag_loss",
             "avg_dagness_node_loss", "avg_combo_loss"]


class ParamSnapshot:
    """``best_model`` of fit() on the fused path: the parameters (and BatchNorm buffers) at the
    best epoch as copies of the engine's two packed parameter buffers, instead of the reference's
    ``copy.deepcopy(self)`` every improving epoch (...withStateSmoothing.py:1553-1559), which
    costs more than the epoch's training steps.  ``materialize()`` builds the module the reference
    would hold (checkpoints); ``restore_into`` is restore_parameters (parameters only)."""

    def __init__(self, model):
        eng = model.engine()
        eng.ensure_bound()
        self.model = model
        with torch.no_grad():
            self.emb = eng.emb.clone()
            self.fac = eng.fac.clone()
            bn = eng.dgcnn.BN1
            self.bn = (bn.running_mean.clone(), bn.running_var.clone(), bn.num_batches_tracked.clone())

    def _slices(self, model):
        """name -> (flat buffer, offset, numel) of every packed parameter of `model` (the fit's model)."""
        eng = model.engine()
        out = {}
        for name, prm in model.named_parameters():
            for base, flat in ((eng.emb, self.emb), (eng.fac, self.fac)):
                off = (prm.data_ptr() - base.data_ptr()) // 4
                if 0 <= off < base.numel() and prm.device == base.device:
                    out[name] = (flat, off, prm.numel())
                    break
        return out

    def restore_into(self, model):
        eng = model.engine()
        eng.ensure_bound()
        with torch.no_grad():
            eng.emb.copy_(self.emb)
            eng.fac.copy_(self.fac)
        eng.invalidate()  # A changed: the Chebyshev supports are recomputed before the next use

    def materialize(self):
        m = copy.deepcopy(self.model)
        sl = self._slices(self.model)
        with torch.no_grad():
            for name, prm in m.named_parameters():
                flat, off, n = sl[name]
                prm.copy_(flat[off:off + n].view_as(prm))
            bn = m.factor_score_embedder.dgcnn.dgcnn.BN1
            bn.running_mean.copy_(self.bn[0])
            bn.running_var.copy_(self.bn[1])
            bn.num_batches_tracked.copy_(self.bn[2])
        return m


def _best_model(model, fused):
    return ParamSnapshot(model) if fused else copy.deepcopy(model)


def _as_module(best_model):
    return best_model.materialize() if isinstance(best_model, ParamSnapshot) else best_model


def restore_parameters(model, best_model):
    """general_utils/model_utils.py:309-313: parameters only, not buffers."""
    if isinstance(best_model, ParamSnapshot):
        best_model.restore_into(model)
        return
    for params, best_params in zip(model.parameters(), best_model.parameters()):
        params.data = best_params


def _confusion(cm):
    from .redcliff_s_cmlp_withStateSmoothing import _confusion_rates
    return _confusion_rates(cm)


def run_fit(model, save_dir, X_train, oA, oB, output_length, max_iter, X_val, lookback, check_every, verbose, GC,
            deltaConEps, in_degree_coeff, out_degree_coeff, prior_factors_path, sc_forecast, sc_factor, sc_cos,
            save_plots):
    if "Freeze" in model.training_mode:
        raise NotImplementedError("Freeze* training modes are not on the fused path")
    if prior_factors_path is not None:
        raise NotImplementedError("prior-initialised factors (prior_factors_path) are not on the fused path")
    if output_length != 1:
        raise NotImplementedError("output_length must be 1")
    fused = model.fused_supported()
    eng = model.engine() if fused else None
    nsup, K, p = model.num_supervised_factors, model.num_factors_nK, model.num_chans
    thresholds = [0.0]
    h = dict((k, []) for k in HIST_KEYS)
    f1_hist = {t: [[] for _ in range(nsup)] for t in thresholds}
    f1_off = {t: [[] for _ in range(nsup)] for t in thresholds}
    roc_hist = {t: [[] for _ in range(nsup)] for t in thresholds}
    roc_off = {t: [[] for _ in range(nsup)] for t in thresholds}
    cm_train = dict((k, []) for k in ("acc", "tpr", "tnr", "fpr", "fnr"))
    cm_val = dict((k, []) for k in ("acc", "tpr", "tnr", "fpr", "fnr"))
    l1_hist = [[] for _ in range(nsup)]
    cos_hist = {"%dand%d" % (i, j): [] for i in range(nsup) for j in range(nsup) if i < j}
    cos_unsup = {"%dand%d" % (i, j): [] for i in range(nsup, K) for j in range(nsup, K) if i < j}
    dc_hist = [[] for _ in range(nsup)]
    dcdd_hist = [[] for _ in range(nsup)]
    daff_hist = [[] for _ in range(nsup)]
    plm_hist = {pl: [[] for _ in range(nsup)] for pl in range(1, p)}
    best_it, best_loss, best_model, iter_start = None, np.inf, None, 0

    if hasattr(model, "chkpt_best_it"):  # resume_training_from_checkpoint was called
        best_model = _best_model(model, fused)
        iter_start = model.chkpt_best_it + 1
        for k in HIST_KEYS:
            h[k] = list(getattr(model, "chkpt_" + k))[:iter_start]
        best_loss, best_it = model.chkpt_best_loss, model.chkpt_best_it

    if fused:
        train = eng.cache_dataset(X_train)
        val = eng.cache_dataset(X_val)
        d_train = eng.workspace(max(train["Bmax"], val["Bmax"]), train["T"])
    Lm = model.Lmax

    for it in range(iter_start, max_iter):
        if verbose:
            print("REDCLIFF_S_CMLP_withStateSmoothing.fit: now on epoch it == ", it, flush=True)
        kinds = phase_of_epoch(model, it)
        if not fused:  # generic path: the reference's batch loop (...withStateSmoothing.py:1331-1364)
            cm = np.zeros((max(nsup, 1), max(nsup, 1)))
            for bi, (Xb, Yb) in enumerate(X_train):
                model.batch_update(it, bi, Xb, Yb, oA, oB, output_length,
                                   running_factor_score_confusion_matrix=cm if nsup > 0 else None)
        else:
            eng.conf.zero_()
            d_train = eng.workspace(train["Bmax"], train["T"])
        if not fused:
            pass
        elif len(kinds) == 1:
            eng.run_steps(kinds, train["X"], train["lab"], train["stats"], d_train, train["rows"], train["sizes"], oA, oB)
        else:  # several updates per batch: batch-major order as in batch_update
            F2 = train["stats"].shape[1] * train["stats"].shape[2]
            for bi, (r, s) in enumerate(zip(train["rows"], train["sizes"])):
                for kind in kinds:
                    eng.run_steps([kind], train["X"], train["lab"], train["stats"][bi:bi + 1], d_train, [r], [s],
                                  oA, oB)
            del F2
        model._set_module_modes(kinds[-1] if kinds else None)
        if nsup > 0:
            if fused:
                cm = eng.conf.cpu().numpy().reshape(nsup, nsup)
            TPR, TNR, FPR, FNR, ACC = _confusion(cm)
            for key, v in zip(("acc", "tpr", "tnr", "fpr", "fnr"), (ACC, TPR, TNR, FPR, FNR)):
                cm_train[key].append(v)

        # ---- GC progress on the first validation batch (:1366-1414)
        model.factor_score_embedder.eval()
        for f in model.factors:
            f.eval()
        if fused:
            nfirst = int(val["sizes"][0])
            Xv = val["X"][:min(nfirst, model.MAX_NUM_SAMPS_FOR_GC_PROGRESS_TRACKING), :Lm, :]
        else:
            Xv = X_val[0][0][:model.MAX_NUM_SAMPS_FOR_GC_PROGRESS_TRACKING, :Lm, :].to(model._device(), torch.float32)
        # conditional GC modes on the fused path: estimates as stacked device tensors, metrics on
        # the GPU (rc_metrics.hip); otherwise the host loops of the reference
        dev_metrics = (fused and 2 <= p <= 64 and model.primary_gc_est_mode in (
            "conditional_factor_exclusive", "conditional_factor_fixed_embedder"))
        with torch.no_grad():
            if dev_metrics:
                mode = model.primary_gc_est_mode
                est_t = model._conditional_gc_stack(mode, Xv[:nsup], False, False, False)
                nolag_np = model._conditional_gc_stack(mode, Xv, False, True, True).cpu().numpy()
                est_host = est_t.cpu().numpy()
                est_np = [[est_host[s, k] for k in range(est_host.shape[1])] for s in range(est_host.shape[0])]
            else:
                est = model.GC(model.primary_gc_est_mode, X=Xv, threshold=False, ignore_lag=False)[:nsup]
                est_np = [[g.detach().cpu().numpy() for g in row] for row in est]
                nolag = model.GC(model.primary_gc_est_mode, X=Xv, threshold=False, ignore_lag=True,
                                 combine_wavelet_representations=True)
                nolag_np = np.stack([np.stack([g.detach().cpu().numpy() for g in row]) for row in nolag])
        if GC is not None and nsup > 0:
            if dev_metrics and len(est_np) > 0:
                vals = M.gc_progress_values(GC, est_t, deltaConEps, in_degree_coeff, out_degree_coeff)
                f1_hist, roc_hist = M.track_roc_stats_from_values(vals, f1_hist, roc_hist, False)
                f1_off, roc_off = M.track_roc_stats_from_values(vals, f1_off, roc_off, True)
                dc_hist, dcdd_hist, daff_hist, plm_hist = M.track_deltacon_stats_from_values(
                    vals, p, dc_hist, dcdd_hist, daff_hist, plm_hist)
            else:
                f1_hist, roc_hist = M.track_roc_stats(GC, est_np, f1_hist, roc_hist, remove_self_connections=False)
                f1_off, roc_off = M.track_roc_stats(GC, est_np, f1_off, roc_off, remove_self_connections=True)
                dc_hist, dcdd_hist, daff_hist, plm_hist = M.track_deltacon_stats(
                    GC, est_np, p, dc_hist, dcdd_hist, daff_hist, plm_hist, deltaConEps, in_degree_coeff,
                    out_degree_coeff)
        if nsup > 0:
            _, l1_hist = M.track_l1_stats(est_np, l1_hist)
        cos_hist = M.track_cosine_stats_batched(nolag_np[:, :nsup], cos_hist, label_offset=0)
        cos_unsup = M.track_cosine_stats_batched(nolag_np[:, nsup:], cos_unsup, label_offset=nsup)

        # ---- validation (:1416-1480)
        if nsup > 0:
            vals = model.validate_training(X_val, output_length, model.num_series, [], [], [], [], [])
            for key, v in zip(("acc", "tpr", "tnr", "fpr", "fnr"), vals[-5:]):
                cm_val[key] = v
            vals = vals[:-5]
        else:
            vals = model.validate_training(X_val, output_length, model.num_series)
        vals = list(vals)
        if not model._WITH_SMOOTHING:
            vals = vals[:4] + [0.0] + vals[4:]
        for k, v in zip(HIST_KEYS, vals):
            h[k].append(v)
        v_forecast, v_factor = vals[0], vals[1]

        # ---- early stopping (:1482-1559)
        if it >= model.num_pretrain_epochs + model.num_acclimation_epochs:
            with np.errstate(all="ignore"):
                cos_mean = np.mean([cos_hist[key][-1] for key in cos_hist.keys()]) if cos_hist else np.nan
            if nsup > 0:
                crit = sc_factor * v_factor + sc_forecast * v_forecast + (sc_cos * cos_mean if nsup > 1 else 0.)
            else:
                crit = sc_forecast * v_forecast
            if crit < best_loss:
                best_loss, best_it, best_model = crit, it, _best_model(model, fused)
            elif (it - best_it) == lookback * check_every:
                if verbose:
                    print("Stopping early")
                break
        else:
            best_it, best_model = it, _best_model(model, fused)

        if it % check_every == 0 and save_dir is not None:
            save_checkpoint(model, save_dir, it, _as_module(best_model), *[h[k] for k in HIST_KEYS], best_loss, best_it, f1_hist,
                            f1_off, roc_hist, roc_off, l1_hist, cos_hist, cos_unsup, dc_hist, dcdd_hist, daff_hist,
                            plm_hist, GC, X_val, cm_train=cm_train, cm_val=cm_val, save_plots=save_plots)

    restore_parameters(model, best_model)
    if save_dir is not None:
        torch.save(model, os.path.join(save_dir, "final_best_model.bin"))
    if nsup > 0:
        final = model.validate_training(X_val, output_length, model.num_series, [], [], [], [], [])
        final_combo = final[-6]
    else:
        final_combo = model.validate_training(X_val, output_length, model.num_series)[-1]
    if verbose:
        print("FINAL BEST (STOPPING CRITERIA) LOSS == ", best_loss, flush=True)
        print("FINAL BEST (STOPPING CRITERIA) EPOCH == ", best_it, flush=True)
        print("FINAL VALIDATION COMBO LOSS == ", final_combo, flush=True)
    model.fit_history = dict(h, best_loss=best_loss, best_it=best_it, f1score_histories=f1_hist,
                             f1score_OffDiag_histories=f1_off, roc_auc_histories=roc_hist,
                             roc_auc_OffDiag_histories=roc_off, gc_factor_l1_loss_histories=l1_hist,
                             gc_factor_cosine_sim_histories=cos_hist,
                             gc_factorUnsupervised_cosine_sim_histories=cos_unsup, deltacon0_histories=dc_hist,
                             deltacon0_with_directed_degrees_histories=dcdd_hist, deltaffinity_histories=daff_hist,
                             path_length_mse_histories=plm_hist, factor_score_train_history=cm_train)
    return final_combo


def save_checkpoint(model, save_dir, it, best_model, avg_forecasting_loss, avg_factor_loss,
                    avg_factor_cos_sim_penalty, avg_fw_l1_penalty, avg_fw_smoothing_penalty, avg_adj_penalty,
                    avg_dagness_reg_loss, avg_dagness_lag_loss, avg_dagness_node_loss, avg_combo_loss, best_loss,
                    best_it, f1score_histories, f1score_OffDiag_histories, roc_auc_histories,
                    roc_auc_OffDiag_histories, gc_factor_l1_loss_histories, gc_factor_cosine_sim_histories,
                    gc_factorUnsupervised_cosine_sim_histories, deltacon0_histories,
                    deltacon0_with_directed_degrees_histories, deltaffinity_histories, path_length_mse_histories,
                    GC=None, X_vis=None, cm_train=None, cm_val=None, save_plots=False, **unused):
    """Writes the two files the reference's evaluation scripts and resume logic read
    (...withStateSmoothing.py:936-990).  Plots (general_utils/plotting.py) are out of scope."""
    os.makedirs(save_dir, exist_ok=True)
    torch.save(best_model, os.path.join(save_dir, "final_best_model.bin"))
    cm_train = cm_train or {}
    cm_val = cm_val or {}
    meta = {
        "epoch": it, "avg_forecasting_loss": avg_forecasting_loss, "avg_factor_loss": avg_factor_loss,
        "avg_factor_cos_sim_penalty": avg_factor_cos_sim_penalty, "avg_fw_l1_penalty": avg_fw_l1_penalty,
        "avg_fw_smoothing_penalty": avg_fw_smoothing_penalty, "avg_adj_penalty": avg_adj_penalty,
        "avg_dagness_reg_loss": avg_dagness_reg_loss, "avg_dagness_lag_loss": avg_dagness_lag_loss,
        "avg_dagness_node_loss": avg_dagness_node_loss, "avg_combo_loss": avg_combo_loss, "best_loss": best_loss,
        "best_it": best_it, "f1score_histories": f1score_histories,
        "f1score_OffDiag_histories": f1score_OffDiag_histories, "roc_auc_histories": roc_auc_histories,
        "roc_auc_OffDiag_histories": roc_auc_OffDiag_histories,
        "factor_score_train_acc_history": cm_train.get("acc"), "factor_score_train_tpr_history": cm_train.get("tpr"),
        "factor_score_train_tnr_history": cm_train.get("tnr"), "factor_score_train_fpr_history": cm_train.get("fpr"),
        "factor_score_train_fnr_history": cm_train.get("fnr"), "factor_score_val_acc_history": cm_val.get("acc"),
        "factor_score_val_tpr_history": cm_val.get("tpr"), "factor_score_val_tnr_history": cm_val.get("tnr"),
        "factor_score_val_fpr_history": cm_val.get("fpr"), "factor_score_val_fnr_history": cm_val.get("fnr"),
        "gc_factor_l1_loss_histories": gc_factor_l1_loss_histories,
        "gc_factor_cosine_sim_histories": gc_factor_cosine_sim_histories,
        "gc_factorUnsupervised_cosine_sim_histories": gc_factorUnsupervised_cosine_sim_histories,
        "deltacon0_histories": deltacon0_histories,
        "deltacon0_with_directed_degrees_histories": deltacon0_with_directed_degrees_histories,
        "deltaffinity_histories": deltaffinity_histories, "path_length_mse_histories": path_length_mse_histories,
    }
    with open(os.path.join(save_dir, "training_meta_data_and_hyper_parameters.pkl"), "wb") as f:
        pkl.dump(meta, f)
