"""REDCLIFF-S ``fit`` (models/redcliff_s_cmlp_withStateSmoothing.py:1175-1647) on the fused engine.

Per epoch: one prepared ``redcliff_train_steps`` call runs every batch of the (device-resident)
training set; the embedder confusion matrix accumulates on the GPU; GC progress is tracked on
the first validation batch (<= 40 windows: ONE embedder launch, the group norms, one
broadcast, one metrics launch); validation runs as one more kernel call; early stopping,
best-model snapshots, checkpoints and ``restore_parameters`` follow the reference's rules,
including its parity hazards:
  * stopping is evaluated only after pretrain + acclimation epochs, with an equality test
    ``it - best_it == lookback * check_every``; before that best_model is refreshed every epoch;
  * GC tracking slices the SAMPLE list to num_supervised_factors;
  * restore_parameters restores parameters only (BatchNorm running statistics stay).
The resume typo of the reference (redcliff_s_cmlp.py:1237) is not reproduced.

The per-fit bookkeeping lives in ``FitTracker`` so that a packed grid search
(``ReplicaPack.fit``, redcliff_amd.replicas) applies exactly the same rules to every replica.
"""
import copy
import gc
import os
import pickle as pkl

import numpy as np
import torch

from . import metrics as M
from .engine import phase_of_epoch

HIST_KEYS = ["avg_forecasting_loss", "avg_factor_loss", "avg_factor_cos_sim_penalty", "avg_fw_l1_penalty",
             "avg_fw_smoothing_penalty", "avg_adj_penalty", "avg_dagness_reg_loss", "avg_dagness_lag_loss",
             "avg_dagness_node_loss", "avg_combo_loss"]
CM_KEYS = ("acc", "tpr", "tnr", "fpr", "fnr")
# The reference's epoch loop re-binds these two history lists to [] before every validation
# (...withStateSmoothing.py:1427-1428, redcliff_s_cmlp.py:1415-1416), so they only ever hold the
# last epoch's value -- in fit_history and in every checkpoint (tests/golden/fit_*.npz).
RESET_EACH_EPOCH = ("avg_dagness_lag_loss", "avg_dagness_node_loss")


def standalone_copy(model):
    """deepcopy of `model` whose parameters and buffers are compact clones of their own values.
    A packed replica's parameters are views of the pack's [R][...] storage (and a single fit's
    of its engine's buffers); a plain deepcopy / torch.save would carry the whole storage."""
    memo = {}
    with torch.no_grad():
        for prm in model.parameters():
            memo[id(prm)] = torch.nn.Parameter(prm.detach().clone(), requires_grad=prm.requires_grad)
        for buf in model.buffers():
            memo[id(buf)] = buf.detach().clone()
    return copy.deepcopy(model, memo)


class ParamSnapshot:
    """``best_model`` of fit() on the fused path: the parameters (and BatchNorm buffers) at the
    best epoch as copies of the engine's two packed parameter buffers, instead of the reference's
    ``copy.deepcopy(self)`` every improving epoch (...withStateSmoothing.py:1553-1559), which
    costs more than the epoch's training steps.  ``materialize()`` builds the module the reference
    would hold (checkpoints); ``restore_into`` is restore_parameters (parameters only)."""

    def __init__(self, model, emb=None, fac=None, bn=None):
        self.model = model
        if emb is not None and fac is not None and bn is not None:  # rows a packed fit keeps (replicas._PackBest)
            self.emb, self.fac, self.bn = emb, fac, bn
            return
        eng = model.engine()
        eng.ensure_bound()  # copies of the live buffers: bindings must be current
        with torch.no_grad():
            self.emb = eng.emb.clone() if emb is None else emb
            self.fac = eng.fac.clone() if fac is None else fac
            if bn is None:
                b = eng.dgcnn.BN1
                bn = (b.running_mean.clone(), b.running_var.clone(), b.num_batches_tracked.clone())
            self.bn = bn

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
        m = standalone_copy(self.model)
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


def _compact_optimizer_state(opt):
    """opt.state_dict() with every tensor cloned: the engine's Adam moments are views of its
    (or a pack's) flat buffers, which must not be serialised whole."""
    sd = opt.state_dict()
    sd["state"] = dict((k, dict((kk, vv.detach().clone() if torch.is_tensor(vv) else vv) for kk, vv in v.items()))
                       for k, v in sd["state"].items())
    return sd


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


class FitTracker:
    """Histories and stopping rule of ONE fit (...withStateSmoothing.py:1316-1559,
    general_utils/model_utils.py:18-209 trackers).  Fed once per epoch with the train confusion
    matrix, the GC-progress inputs and the validation values; decides improve / stop."""

    def __init__(self, model, GC, deltaConEps, in_degree_coeff, out_degree_coeff, sc_forecast, sc_factor, sc_cos,
                 lookback, check_every):
        self.model = model
        self.GC = GC
        self.eps, self.cin, self.cout = deltaConEps, in_degree_coeff, out_degree_coeff
        self.sc_forecast, self.sc_factor, self.sc_cos = sc_forecast, sc_factor, sc_cos
        self.lookback, self.check_every = lookback, check_every
        nsup, K, p = model.num_supervised_factors, model.num_factors_nK, model.num_chans
        self.nsup, self.K, self.p = nsup, K, p
        thresholds = [0.0]
        self.h = dict((k, []) for k in HIST_KEYS)
        self.f1_hist = {t: [[] for _ in range(nsup)] for t in thresholds}
        self.f1_off = {t: [[] for _ in range(nsup)] for t in thresholds}
        self.roc_hist = {t: [[] for _ in range(nsup)] for t in thresholds}
        self.roc_off = {t: [[] for _ in range(nsup)] for t in thresholds}
        self.cm_train = dict((k, []) for k in CM_KEYS)
        self.cm_val = dict((k, []) for k in CM_KEYS)
        self.l1_hist = [[] for _ in range(nsup)]
        self.cos_hist = {"%dand%d" % (i, j): [] for i in range(nsup) for j in range(nsup) if i < j}
        self.cos_unsup = {"%dand%d" % (i, j): [] for i in range(nsup, K) for j in range(nsup, K) if i < j}
        self.dc_hist = [[] for _ in range(nsup)]
        self.dcdd_hist = [[] for _ in range(nsup)]
        self.daff_hist = [[] for _ in range(nsup)]
        self.plm_hist = {pl: [[] for _ in range(nsup)] for pl in range(1, p)}
        self.best_it, self.best_loss, self.best_model, self.iter_start = None, np.inf, None, 0
        self.stopped_at = None

    def resume(self, fused):
        """resume_training_from_checkpoint was called (...withStateSmoothing.py:1229-1277)."""
        m = self.model
        if not hasattr(m, "chkpt_best_it"):
            return 0
        self.best_model = _best_model(m, fused)
        self.iter_start = m.chkpt_best_it + 1
        for k in HIST_KEYS:
            self.h[k] = list(getattr(m, "chkpt_" + k))[:self.iter_start]
        self.best_loss, self.best_it = m.chkpt_best_loss, m.chkpt_best_it
        return self.iter_start

    def train_confusion(self, cm):
        if self.nsup > 0:
            TPR, TNR, FPR, FNR, ACC = _confusion(cm)
            for key, v in zip(CM_KEYS, (ACC, TPR, TNR, FPR, FNR)):
                self.cm_train[key].append(v)

    def gc_progress(self, est_np, nolag_np, vals):
        """est_np: [nsup samples][K] lagged estimates (host); nolag_np (S, K, p, p, 1) lag-free
        combined estimates; vals: device metric values (S, G, 6 + p) or None (host trackers)."""
        GC, nsup = self.GC, self.nsup
        if GC is not None and nsup > 0:
            if vals is not None:
                if len(est_np) > 0:
                    self.f1_hist, self.roc_hist = M.track_roc_stats_from_values(vals, self.f1_hist, self.roc_hist, False)
                    self.f1_off, self.roc_off = M.track_roc_stats_from_values(vals, self.f1_off, self.roc_off, True)
                    self.dc_hist, self.dcdd_hist, self.daff_hist, self.plm_hist = M.track_deltacon_stats_from_values(
                        vals, self.p, self.dc_hist, self.dcdd_hist, self.daff_hist, self.plm_hist)
            else:
                self.f1_hist, self.roc_hist = M.track_roc_stats(GC, est_np, self.f1_hist, self.roc_hist,
                                                                remove_self_connections=False)
                self.f1_off, self.roc_off = M.track_roc_stats(GC, est_np, self.f1_off, self.roc_off,
                                                              remove_self_connections=True)
                self.dc_hist, self.dcdd_hist, self.daff_hist, self.plm_hist = M.track_deltacon_stats(
                    GC, est_np, self.p, self.dc_hist, self.dcdd_hist, self.daff_hist, self.plm_hist, self.eps,
                    self.cin, self.cout)
        if nsup > 0:
            _, self.l1_hist = M.track_l1_stats(est_np, self.l1_hist)
        self.cos_hist = M.track_cosine_stats_batched(nolag_np[:, :nsup], self.cos_hist, label_offset=0)
        self.cos_unsup = M.track_cosine_stats_batched(nolag_np[:, nsup:], self.cos_unsup, label_offset=nsup)

    def validation(self, vals):
        """The tuple validate_training returns (with 5 one-entry confusion histories when supervised)."""
        if self.nsup > 0:
            for key, v in zip(CM_KEYS, vals[-5:]):
                self.cm_val[key] = v
            vals = vals[:-5]
        vals = list(vals)
        if not self.model._WITH_SMOOTHING:
            vals = vals[:4] + [0.0] + vals[4:]
        for k, v in zip(HIST_KEYS, vals):
            if k in RESET_EACH_EPOCH:
                self.h[k] = []
            self.h[k].append(v)
        self._vf, self._vfac = vals[0], vals[1]

    def past_warmup(self, it):
        """Epoch `it` is past pretraining and acclimation: the stopping rule applies (:1483)."""
        m = self.model
        return it >= m.num_pretrain_epochs + m.num_acclimation_epochs

    def may_stop(self, it):
        """step(it) can return True only when this holds (the fit can stop at `it` only past the
        warm-up and exactly lookback * check_every epochs after its best epoch, :1549-1559).  The
        packed fit asks it before epoch `it` is decided, to skip saving the Adam moments when no
        replica can be rolled back; step() itself decides through the same test."""
        return self.past_warmup(it) and self.best_it is not None and \
            (it - self.best_it) == self.lookback * self.check_every

    def step(self, it, snapshot):
        """Early stopping (:1482-1559).  snapshot() makes the best-model copy; returns True when
        the fit stops at this epoch."""
        m = self.model
        if self.past_warmup(it):
            with np.errstate(all="ignore"):
                cos_mean = np.mean([self.cos_hist[key][-1] for key in self.cos_hist.keys()]) if self.cos_hist else np.nan
            if "Freeze" in m.training_mode:  # :1486-1491; raises as the reference's does
                m.determine_which_factors_need_updates(self.best_model, [True] * self.K)
                raise AssertionError("unreachable: the reference's Freeze decision cannot complete")
            if self.nsup > 0:
                crit = self.sc_factor * self._vfac + self.sc_forecast * self._vf + (
                    self.sc_cos * cos_mean if self.nsup > 1 else 0.)
            else:
                crit = self.sc_forecast * self._vf
            if crit < self.best_loss:
                self.best_loss, self.best_it, self.best_model = crit, it, snapshot()
            elif self.may_stop(it):
                self.stopped_at = it
                return True
        else:
            self.best_it, self.best_model = it, snapshot()
        return False

    def checkpoint(self, save_dir, it, optimizers=None, save_plots=False):
        save_checkpoint(self.model, save_dir, it, _as_module(self.best_model), *[self.h[k] for k in HIST_KEYS],
                        self.best_loss, self.best_it, self.f1_hist, self.f1_off, self.roc_hist, self.roc_off,
                        self.l1_hist, self.cos_hist, self.cos_unsup, self.dc_hist, self.dcdd_hist, self.daff_hist,
                        self.plm_hist, self.GC, None, cm_train=self.cm_train, cm_val=self.cm_val,
                        save_plots=save_plots, optimizers=optimizers)

    def history(self):
        return dict(self.h, best_loss=self.best_loss, best_it=self.best_it, f1score_histories=self.f1_hist,
                    f1score_OffDiag_histories=self.f1_off, roc_auc_histories=self.roc_hist,
                    roc_auc_OffDiag_histories=self.roc_off, gc_factor_l1_loss_histories=self.l1_hist,
                    gc_factor_cosine_sim_histories=self.cos_hist,
                    gc_factorUnsupervised_cosine_sim_histories=self.cos_unsup, deltacon0_histories=self.dc_hist,
                    deltacon0_with_directed_degrees_histories=self.dcdd_hist,
                    deltaffinity_histories=self.daff_hist, path_length_mse_histories=self.plm_hist,
                    factor_score_train_history=self.cm_train, stopped_at=self.stopped_at)


def _per_graph_appends(hists, run, n, G):
    """The length rules of model_utils.py:63-84 / :136-158 for one fit's per-graph histories
    (len(hists) = nsup lists) given its per-graph running sums run[G]: returns the values to
    append and whether the lengths match (only then are the path-length histories appended)."""
    L = len(hists)
    if L != G:
        if G == 1 and L > 1:
            return [run[0] / n] * L, False
        assert L < G
    return [run[i] / n for i in range(L)], L == G


def confusion_rates_many(cms):
    """_confusion_rates of a stack of confusion matrices [Ra][n][n] (integer counts, so every sum
    is exact in any order): (TPR, TNR, FPR, FNR, ACC), each [Ra][n]."""
    cm = np.asarray(cms, dtype=np.float64)
    TP = np.diagonal(cm, axis1=1, axis2=2)
    FP = cm.sum(axis=1) - TP
    FN = cm.sum(axis=2) - TP
    TN = cm.sum(axis=(1, 2))[:, None] - (FP + FN + TP)
    with np.errstate(divide="ignore", invalid="ignore"):
        return TP / (TP + FN), TN / (TN + FP), FP / (FP + TN), FN / (TP + FN), (TP + TN) / (TP + FP + FN + TN)


def train_confusion_many(trackers, cms, log=None, cols=None):
    """FitTracker.train_confusion of several fits (cms [Ra][nsup][nsup] integer counts): the
    confusion rates of all of them in one vectorised pass (exact: integer-valued sums).  log: a
    DeferredHistories that holds the rates until its flush (nothing reads cm_train mid-fit)."""
    if not trackers or trackers[0].nsup <= 0:
        return
    TPR, TNR, FPR, FNR, ACC = confusion_rates_many(cms)
    if log is not None:
        log.add_confusion(trackers, np.stack([ACC, TPR, TNR, FPR, FNR], axis=1), cols)
        return
    for i, t in enumerate(trackers):
        for key, v in zip(CM_KEYS, (ACC, TPR, TNR, FPR, FNR)):
            t.cm_train[key].append(v[i].copy())


def _extend_per_graph(hists, cols, G):
    """_per_graph_appends over a stack of epochs: cols = the epochs' run / n as G python lists
    (graph-major); returns whether the lengths match."""
    L = len(hists)
    if L != G:
        if G == 1 and L > 1:
            for h in hists:
                h.extend(cols[0])
            return False
        assert L < G
    for j in range(L):
        hists[j].extend(cols[j])
    return L == G


def _stack_log(entries, pick):
    """Entries [(trackers, cols, arrays...)] of a DeferredHistories log as one [E][T][...] array
    (T = the fits, by their column -- the pack's replica index, or order of first appearance;
    NaN where a fit was not active) plus, per fit, its epoch rows (a slice when they are
    consecutive, as a pack's always are)."""
    order, colof, bycol = [], {}, {}
    for e in entries:
        if e[1] is None:
            for t in e[0]:
                if id(t) not in colof:
                    colof[id(t)] = len(order)
                    order.append(t)
        else:
            bycol.update(zip(e[1], e[0]))
    if bycol:
        order = [bycol.get(c) for c in range(max(bycol) + 1)]
    first = next(pick(e) for e in entries if pick(e) is not None)
    V = np.full((len(entries), len(order)) + first.shape[1:], np.nan, dtype=first.dtype)
    present = np.zeros((len(entries), len(order)), dtype=bool)
    for i, e in enumerate(entries):
        a = pick(e)
        if a is None:
            continue
        cols = e[1] if e[1] is not None else [colof[id(t)] for t in e[0]]
        V[i, cols] = a
        present[i, cols] = True
    rows = []
    for j in range(len(order)):
        idx = np.flatnonzero(present[:, j])
        if idx.size and idx[-1] - idx[0] + 1 == idx.size:
            rows.append(slice(int(idx[0]), int(idx[-1]) + 1))
        else:
            rows.append(idx)
    return V, order, rows


class DeferredHistories:
    """The per-epoch history appends of a packed fit that no decision of the fit reads -- the
    GC-progress histories (f1 / ROC / DeltaCon / path-length / factor-L1) and the train confusion
    rates -- logged as arrays per epoch and appended to every fit's tracker lists at flush(): the
    same values in the same order as gc_progress_many / train_confusion_many append them each
    epoch (the cosine-similarity histories, which the stopping rule reads, stay per epoch).
    flush() stacks the log into [epoch][fit][...] arrays, divides once, and extends each history
    list with its fit's column -- one list extend per (fit, history) instead of one python append
    per (fit, history, epoch).  The packed fit flushes before every checkpoint and at the end."""

    def __init__(self):
        self.gc, self.cm = [], []

    def add_gc(self, trackers, run, n, l1m, cols=None):
        """cols: the fits' fixed column indices (a pack's replica indices), else by first appearance."""
        self.gc.append((list(trackers), None if cols is None else list(cols), run, float(n), l1m))

    def add_confusion(self, trackers, rates, cols=None):
        self.cm.append((list(trackers), None if cols is None else list(cols), rates))

    def flush(self):
        if any(e[2] is not None for e in self.gc):
            V, order, rows = _stack_log(self.gc, lambda e: e[2])  # [E][T][G][6 + p] running sums
            n = np.asarray([e[3] for e in self.gc], dtype=np.float64)
            W = V / n[:, None, None, None]  # run / n, as the per-epoch appends divide
            G, pv = W.shape[2], W.shape[3] - 6
            for j, (t, rw) in enumerate(zip(order, rows)):
                if t is None:
                    continue
                cols = np.transpose(W[rw, j], (2, 1, 0)).tolist()  # [6 + p][G][E] python floats
                for c, f1h, roch in ((0, t.f1_hist, t.roc_hist), (2, t.f1_off, t.roc_off)):
                    for thresh in f1h.keys():
                        _extend_per_graph(f1h[thresh], cols[c], G)
                        _extend_per_graph(roch[thresh], cols[c + 1], G)
                full = _extend_per_graph(t.dc_hist, cols[4], G)
                _extend_per_graph(t.dcdd_hist, cols[5], G)
                _extend_per_graph(t.daff_hist, cols[6], G)
                if full:
                    for pl in range(1, min(t.p, pv)):
                        for g in range(len(t.dc_hist)):
                            t.plm_hist[pl][g].extend(cols[6 + pl][g])
        if any(e[4] is not None for e in self.gc):
            V, order, rows = _stack_log(self.gc, lambda e: e[4])  # [E][T][K] factor-L1 means
            for j, (t, rw) in enumerate(zip(order, rows)):
                if t is None:
                    continue
                X = V[rw, j].T.tolist()
                for k in range(len(t.l1_hist)):
                    t.l1_hist[k].extend(X[k])
        if self.cm:
            V, order, rows = _stack_log(self.cm, lambda e: e[2])  # [E][T][5][nsup] confusion rates
            for j, (t, rw) in enumerate(zip(order, rows)):
                if t is None:
                    continue
                C = np.array(V[rw, j])  # one private array per fit: its rows are the appended vectors
                for k, key in enumerate(CM_KEYS):
                    t.cm_train[key].extend(list(C[:, k]))
        self.gc, self.cm = [], []


def gc_progress_many(trackers, vals, l1, nrm, dots, log=None, cols=None):
    """FitTracker.gc_progress (device-metrics path) of several fits at once -- a packed grid search
    updates every replica's trackers in a few array operations instead of R python loops.

    vals (Ra, S, G, 6 + p) device metric values (redcliff_gc_progress) or None; l1 (Ra, S, K),
    nrm (Ra, Sn, K), dots (Ra, Sn, K, K): the per-estimate statistics of metrics.gc_track_values
    (device) or metrics.track_values_host; trackers share GC, nsup, K and p.  With the host
    statistics every appended value is bit-identical to the per-fit trackers' (metrics.track_*):
    the reference's python-float running sums over samples are left-to-right float64 cumulative
    sums, the history length rules are model_utils.py:63-84 / :136-158.  log: a DeferredHistories
    that takes every history but the cosine ones until its flush (cols: the fits' columns there)."""
    t0 = trackers[0]
    GC, nsup, K = t0.GC, t0.nsup, t0.K
    S = l1.shape[1]
    run, n = None, float(S)
    if GC is not None and nsup > 0 and vals is not None and S > 0:
        run = np.cumsum(vals, axis=1)[:, -1]  # (Ra, G, C): _running over samples
        for hist in (t0.f1_hist, t0.f1_off):
            if any(thresh != 0.0 for thresh in hist.keys()):
                raise ValueError("device GC-progress metrics cover the fit's threshold 0.0 only")
    l1m = None
    if nsup > 0:  # track_l1_stats over every (sample, factor) estimate
        if S == 0:
            raise IndexError("list index out of range")  # track_l1_stats on an empty sample list
        l1m = np.cumsum(l1, axis=1)[:, -1] / float(S)  # (Ra, K)
    if log is not None:
        log.add_gc(trackers, run, n, l1m, cols)
    else:
        if run is not None:
            G = run.shape[1]
            pv = vals.shape[3] - 6
            for i, t in enumerate(trackers):
                for col, f1h, roch in ((0, t.f1_hist, t.roc_hist), (2, t.f1_off, t.roc_off)):
                    for thresh in f1h.keys():
                        f1v, _ = _per_graph_appends(f1h[thresh], run[i, :, col].tolist(), n, G)
                        rov, _ = _per_graph_appends(roch[thresh], run[i, :, col + 1].tolist(), n, G)
                        for j in range(len(f1h[thresh])):
                            f1h[thresh][j].append(f1v[j])
                            roch[thresh][j].append(rov[j])
                ri = run[i].tolist()
                dcv, full = _per_graph_appends(t.dc_hist, [r[4] for r in ri], n, G)
                dddv, _ = _per_graph_appends(t.dcdd_hist, [r[5] for r in ri], n, G)
                dafv, _ = _per_graph_appends(t.daff_hist, [r[6] for r in ri], n, G)
                for j in range(len(t.dc_hist)):
                    t.dc_hist[j].append(dcv[j])
                    t.dcdd_hist[j].append(dddv[j])
                    t.daff_hist[j].append(dafv[j])
                    if full:
                        for pl in range(1, min(t.p, pv)):
                            t.plm_hist[pl][j].append(ri[j][6 + pl] / n)
        if l1m is not None:
            for i, t in enumerate(trackers):
                li = l1m[i].tolist()
                for j in range(len(t.l1_hist)):
                    t.l1_hist[j].append(li[j])
    Ra, Sn = dots.shape[0], dots.shape[1]
    for lo, hi, attr in ((0, nsup, "cos_hist"), (nsup, K, "cos_unsup")):  # track_cosine_stats_batched
        if hi - lo < 2 or Sn == 0:
            continue
        nr = nrm[:, :, lo:hi]
        nr = np.where(np.isfinite(nr), nr, -1.)
        nr = np.maximum(nr, 1e-8)
        for i1 in range(hi - lo):
            for i2 in range(i1 + 1, hi - lo):
                cv = dots[:, :, lo + i1, lo + i2] / (nr[:, :, i1] * nr[:, :, i2])
                tot = np.cumsum(np.concatenate([np.zeros((Ra, 1)), cv], axis=1), axis=1)[:, -1] / float(Sn)
                key = "%dand%d" % (i1 + lo, i2 + lo)
                for i, t in enumerate(trackers):
                    getattr(t, attr)[key].append(float(tot[i]))


def conditional_gc_estimates(w, G, G0, A, nsup, ls, mode):
    """The two GC-progress estimate stacks of fit() (:1366-1414) from the embedder weights
    w (..., S, K) (post-sigmoid), the factor group norms G (..., K, p, p, L) / G0 (..., K, p, p)
    and A (..., p, p) -- leading dims are replicas for a packed fit.  Element-wise the same
    operations as GC(mode, X, threshold=False) (the reference's per-(sample, factor) products):
      est   = lagged estimates of the first nsup samples, no abs on A   (..., nsup, K, p, p, ls)
      nolag = lag-free estimates of all samples, combine=True (|A|)     (..., S, K, p, p, 1)."""
    eg = A.transpose(-1, -2).unsqueeze(-1)  # (..., p, p, 1): DGCNN GC = A^T (models/dgcnn.py:47-61)
    egc = torch.abs(A).transpose(-1, -2).unsqueeze(-1)
    ws = w[..., :nsup, :, None, None, None]
    wa = w[..., :, :, None, None, None]
    est = ws * G.unsqueeze(-5)
    nolag = wa * G0.unsqueeze(-1).unsqueeze(-5)
    if mode == "conditional_factor_fixed_embedder":
        est = est[..., -ls:] + eg.unsqueeze(-4).unsqueeze(-4)[..., -ls:]
        nolag = nolag + egc.unsqueeze(-4).unsqueeze(-4)
    return est, nolag


def run_fit(*args, **kw):
    """fit() on the fused engine (see _run_fit).  The host side of an epoch is python; the cyclic
    garbage collector is paused for the fit (restored afterwards): its full passes over the model's
    module tree land inside epochs."""
    gc_was = gc.isenabled()
    gc.disable()
    try:
        return _run_fit(*args, **kw)
    finally:
        if gc_was:
            gc.enable()


def _eval_modes(model):
    """The module modes every fit epoch ends in: GC tracking and validate_training call .eval() on
    the embedder and every factor (...withStateSmoothing.py:1366-1480)."""
    model.factor_score_embedder.eval()
    for f in model.factors:
        f.eval()


def _train_epoch(model, eng, train, d_train, plans, oA, oB, ep):
    """Enqueue the training steps of epoch `ep` (one prepared launch chain per update kind)."""
    kinds = phase_of_epoch(model, ep)
    eng.conf.zero_()
    if len(kinds) == 1:
        key = kinds[0]
        if key not in plans:
            plans[key] = eng.plan_steps(key, train["X"], train["lab"], train["stats"], d_train, train["rows"],
                                        train["sizes"], oA, oB)
        plans[key].run()
    else:  # several updates per batch: batch-major order as in batch_update
        for bi, (r, s) in enumerate(zip(train["rows"], train["sizes"])):
            for kind in kinds:
                eng.run_steps([kind], train["X"], train["lab"], train["stats"][bi:bi + 1], d_train, [r], [s], oA, oB)


class _SavedState:
    """Everything a training epoch advances in a fused single fit (parameters, Adam moments and
    step counts, BatchNorm statistics), copied on the device before a speculative epoch."""

    def __init__(self, eng):
        self.eng = eng
        self.t = {}
        self.bufs = None

    def _live(self):
        e = self.eng
        bn = e.dgcnn.BN1
        out = [e.emb, e.fac, e.bn, bn.num_batches_tracked]
        for g in ("A", "B"):
            if e.opt[g] is not None:
                out += [e.opt[g]["m"], e.opt[g]["v"]]
        return out

    def save(self):
        live = self._live()
        if self.bufs is None or len(self.bufs) != len(live):
            self.bufs = [torch.empty_like(t) for t in live]
        with torch.no_grad():
            for d, t in zip(self.bufs, live):
                d.copy_(t)
        self.t = dict((g, None if self.eng.opt[g] is None else self.eng.opt[g]["t"]) for g in ("A", "B"))

    def snapshot(self, model):
        """ParamSnapshot (best_model) of the saved state."""
        b = self.bufs
        with torch.no_grad():
            return ParamSnapshot(model, emb=b[0].clone(), fac=b[1].clone(),
                                 bn=(b[2][0].clone(), b[2][1].clone(), b[3].clone()))

    def restore(self):
        e = self.eng
        live = self._live()
        assert len(live) == len(self.bufs), "an optimizer group was bound during the speculative epoch"
        with torch.no_grad():
            for d, t in zip(self.bufs, live):
                t.copy_(d)
        for g, t in self.t.items():
            if t is not None:
                e.opt[g]["t"] = t
        e._sync_steps()
        e.supports_fresh = False
        # a hand-off timeout the undone epoch logged must not fail a later check: its gradients
        # were discarded with it (the word is cleared behind the epoch's launches, same stream)
        e.status_view().zero_()


def _device_epochs(model, eng, tr, train, val, d_train, plans, oA, oB, iter_start, max_iter, save_dir, check_every,
                   verbose, GC, deltaConEps, in_degree_coeff, out_degree_coeff, save_plots, hook, runner=None,
                   writer=True):
    """fit()'s epochs on the fused engine with the per-epoch evaluation on the device.

    Per epoch the training steps are one prepared launch chain; the evaluation (train confusion
    matrix, GC progress on the first validation batch (:1366-1414: one embedder launch, the group
    norms, one broadcast, the metrics and tracker-statistics launches) and validation (:1416-1480,
    batches on the replica axis)) is enqueued behind it and copied back ONCE.  While the host
    digests epoch `it`, the GPU already trains epoch it + 1 (speculatively, state saved first):
    the best-model snapshot of `it` comes from the saved state, and if the fit stops at `it` the
    speculative epoch is undone (_SavedState.restore), so the fit ends exactly where the
    reference's does.  No speculation past max_iter or across a checkpoint epoch.  The launches
    take their BatchNorm mode from flags, so the module flags are set once (_eval_modes)."""
    nsup, p = model.num_supervised_factors, model.num_chans
    Lm, ls = model.Lmax, min(model.gen_lag, model.embed_lag)
    saved = _SavedState(eng)
    if runner is None:
        def train_epoch(ep):
            _train_epoch(model, eng, train, d_train, plans, oA, oB, ep)
    else:
        train_epoch = runner
    freeze = "Freeze" in model.training_mode  # the Freeze decision raises: no epoch runs ahead of it
    it = iter_start
    if it < max_iter:
        hook(it)
        train_epoch(it)
    while it < max_iter:
        if verbose:
            print("REDCLIFF_S_CMLP_withStateSmoothing.fit: now on epoch it == ", it, flush=True)
        with torch.no_grad():
            conf_d = eng.conf.clone()
            nfirst = int(val["sizes"][0])
            Xv = val["X"][:min(nfirst, model.MAX_NUM_SAMPS_FOR_GC_PROGRESS_TRACKING), :Lm, :]
            w, _ = model._labels_from_w(eng.embed_raw(Xv))
            G, G0 = eng.gc_norms()
            est_t, nolag_t = conditional_gc_estimates(w, G, G0, eng.dgcnn.A.detach(), nsup, ls,
                                                      model.primary_gc_est_mode)
            vals_d = None
            if GC is not None and nsup > 0 and est_t.shape[0] > 0:
                vals_d = M.gc_progress_values(GC, est_t, deltaConEps, in_degree_coeff, out_degree_coeff, host=False)
            l1_d, dots_d = M.gc_track_values(est_t, nolag_t, host=False)
            acc_d, confv_d = eng.run_values(val["X"], val["lab"], d_train, val["rows"], val["sizes"], host=False)
            pending = M.fetch_async([conf_d, l1_d, dots_d, acc_d, confv_d, eng.status_view()] +
                                    ([vals_d] if vals_d is not None else []))
        spec = (it + 1 < max_iter and not (save_dir is not None and it % check_every == 0) and not freeze
                and it + 1 not in hook.at)
        if spec:
            saved.save()
            train_epoch(it + 1)
        got = pending.wait()
        cm, l1, dots, accs, confs = got[:5]
        vals = got[6] if vals_d is not None else None
        eng.raise_on_status(got[5], "fit epoch %d" % it)
        tr.train_confusion(cm.reshape(nsup, nsup) if nsup > 0 else None)
        l1, nrm, dots = M.track_values_finish(l1, dots)
        gc_progress_many([tr], None if vals is None else vals[None], l1[None], nrm[None], dots[None])
        acc, confv = eng.values_from_rows(accs, confs)
        hists = [[] for _ in range(5)] if nsup > 0 else [None] * 5
        tr.validation(model._validation_tuple(acc, float(val["len"]), confv, *hists))
        # ---- early stopping (:1482-1559)
        if tr.step(it, (lambda: saved.snapshot(model)) if spec else (lambda: _best_model(model, True))):
            if spec:
                saved.restore()
            if verbose:
                print("Stopping early")
            break
        if it % check_every == 0 and save_dir is not None and writer:
            _eval_modes(model)
            tr.checkpoint(save_dir, it, optimizers=(oA, oB), save_plots=save_plots)
        it += 1
        if not spec and it < max_iter:
            hook(it)
            train_epoch(it)


def _host_epochs(model, eng, tr, fused, train, val, d_train, plans, X_train, X_val, oA, oB, output_length, iter_start,
                 max_iter, save_dir, check_every, verbose, save_plots, hook, runner=None, writer=True):
    """fit()'s epochs when the GC-progress metrics run on the host (the generic path, or GC
    modes / sizes outside the device metrics): the reference's loop (...withStateSmoothing.py:
    1316-1559) with the fused training steps where available."""
    nsup = model.num_supervised_factors
    Lm = model.Lmax
    for it in range(iter_start, max_iter):
        if verbose:
            print("REDCLIFF_S_CMLP_withStateSmoothing.fit: now on epoch it == ", it, flush=True)
        hook(it)
        kinds = phase_of_epoch(model, it)
        if not fused:  # generic path: the reference's batch loop (...withStateSmoothing.py:1331-1364)
            cm = np.zeros((max(nsup, 1), max(nsup, 1)))
            for bi, (Xb, Yb) in enumerate(X_train):
                model.batch_update(it, bi, Xb, Yb, oA, oB, output_length,
                                   running_factor_score_confusion_matrix=cm if nsup > 0 else None)
            model._set_module_modes(kinds[-1] if kinds else None)  # the generic modules read their flags
        else:
            if runner is not None:
                runner(it)
            else:
                _train_epoch(model, eng, train, d_train, plans, oA, oB, it)
            eng.check_device_status("fit epoch %d" % it)
            if nsup > 0:
                cm = eng.conf.cpu().numpy().reshape(nsup, nsup)
        tr.train_confusion(cm if nsup > 0 else None)
        # ---- GC progress on the first validation batch (:1366-1414)
        _eval_modes(model)
        with torch.no_grad():
            if fused:
                Xv = val["X"][:min(int(val["sizes"][0]), model.MAX_NUM_SAMPS_FOR_GC_PROGRESS_TRACKING), :Lm, :]
            else:
                Xv = X_val[0][0][:model.MAX_NUM_SAMPS_FOR_GC_PROGRESS_TRACKING, :Lm, :].to(model._device(),
                                                                                          torch.float32)
            est = model.GC(model.primary_gc_est_mode, X=Xv, threshold=False, ignore_lag=False)[:nsup]
            est_np = [[g.detach().cpu().numpy() for g in row] for row in est]
            nolag = model.GC(model.primary_gc_est_mode, X=Xv, threshold=False, ignore_lag=True,
                             combine_wavelet_representations=True)
            nolag_np = np.stack([np.stack([g.detach().cpu().numpy() for g in row]) for row in nolag])
        tr.gc_progress(est_np, nolag_np, None)
        # ---- validation (:1416-1480)
        if fused:
            tr.validation(model._validate_fused(X_val, nsup > 0))
        elif nsup > 0:
            tr.validation(model.validate_training(X_val, output_length, model.num_series, [], [], [], [], []))
        else:
            tr.validation(model.validate_training(X_val, output_length, model.num_series))
        # ---- early stopping (:1482-1559)
        if tr.step(it, lambda: _best_model(model, fused)):
            if verbose:
                print("Stopping early")
            break
        if it % check_every == 0 and save_dir is not None and writer:
            tr.checkpoint(save_dir, it, optimizers=(oA, oB), save_plots=save_plots)


def _prior_hook(model, X_train, prior):
    """it -> None: the factor re-ordering fit() runs at the start of epoch num_pretrain_epochs
    of the "pretrain_factor" modes (...withStateSmoothing.py:1318-1326)."""
    path, cost, start, nb = prior[:4]
    allow_pickle = prior[4] if len(prior) > 4 else False
    at = set()
    if "pretrain_factor" in model.training_mode:
        at.add(model.num_pretrain_epochs)
    if path is not None:
        at.add(0)

    def hook(it):
        if it in at:
            model.initialize_factors_with_prior(prior_factors_path=path, X_train=X_train, cost_criteria=cost,
                                                unsupervised_start_index=start, max_batches=nb,
                                                allow_pickle=allow_pickle)
    hook.at = at
    return hook


def _freeze_by_batch(model, fused, X_train, oA, oB, output_length, it):
    """The first batch_update of a FreezeByBatch fit (:1331-1342): best_model is the copy fit()
    makes before its loop (:1230), every factor is in training; batch_update's Freeze decision
    raises as the reference's does (determine_which_factors_need_updates)."""
    nsup = model.num_supervised_factors
    cm = np.zeros((nsup, nsup)) if nsup > 0 else None
    for bi, (Xb, Yb) in enumerate(X_train):
        model.batch_update(it, bi, Xb, Yb, oA, oB, output_length, best_model=_best_model(model, fused),
                           training_status_of_each_factor=[True] * model.num_factors_nK,
                           running_factor_score_confusion_matrix=cm)


def _run_fit(model, save_dir, X_train, oA, oB, output_length, max_iter, X_val, lookback, check_every, verbose, GC,
             deltaConEps, in_degree_coeff, out_degree_coeff, prior, sc_forecast, sc_factor, sc_cos,
             save_plots, runner=None, writer=True, train_ds=None):
    """runner(it), when given, trains epoch `it` in place of the fused single-fit epoch (the
    data-parallel fit: redcliff_amd.data_parallel); writer=False: no files (ranks > 0);
    train_ds: the runner's own device copy of the training set (the data-parallel fit's shard
    cache), used in place of caching X_train whole -- a rank then holds only its shards."""
    if output_length != 1:
        raise NotImplementedError("output_length must be 1")
    fused = model.fused_supported()
    eng = model.engine() if fused else None
    nsup = model.num_supervised_factors
    tr = FitTracker(model, GC, deltaConEps, in_degree_coeff, out_degree_coeff, sc_forecast, sc_factor, sc_cos,
                    lookback, check_every)
    iter_start = tr.resume(fused)
    if "Freeze" in model.training_mode:
        if tr.best_model is None:  # fit()'s try block deep-copies the model before the loop (:1230)
            tr.best_model = _best_model(model, fused)
        if "FreezeByBatch" in model.training_mode and iter_start < max_iter:
            _freeze_by_batch(model, fused, X_train, oA, oB, output_length, iter_start)
    hook = _prior_hook(model, X_train, prior)
    ost = getattr(model, "chkpt_optimizer_state", None)
    if ost is not None:  # resume_training_from_checkpoint(..., load_optimizer_state=True)
        oA.load_state_dict(ost["A"])
        oB.load_state_dict(ost["B"])
        if fused:
            eng.opt = {"A": None, "B": None}  # re-bind: the kernels' moment buffers take the loaded state
        del model.chkpt_optimizer_state

    if fused:
        if train_ds is not None and runner is None:
            raise ValueError("train_ds is the runner's training set: pass both or neither")
        train = train_ds if train_ds is not None else eng.cache_dataset(X_train)
        val = eng.cache_dataset(X_val)
        # (a data-parallel runner sizes the workspace for its shards; validation is unsharded)
        d_train = eng.workspace(max(train["Bmax"] if runner is None else 1, val["Bmax"]), train["T"])
        plans = {}

    # The device metrics track num_chans-sized graphs of the uncombined estimates; a wavelet model
    # (num_series = num_chans * (l + 1)) needs the reference's combine_wavelet_representations GC
    # calls (:1396-1407), so it takes the host loop, which makes them (and fails where they fail).
    dev_metrics = (fused and model.wavelet_level is None and 2 <= model.num_series <= 64
                   and model.primary_gc_est_mode in ("conditional_factor_exclusive",
                                                     "conditional_factor_fixed_embedder"))
    if dev_metrics:
        _device_epochs(model, eng, tr, train, val, d_train, plans, oA, oB, iter_start, max_iter, save_dir, check_every,
                       verbose, GC, deltaConEps, in_degree_coeff, out_degree_coeff, save_plots, hook, runner=runner,
                       writer=writer)
    else:
        _host_epochs(model, eng, tr, fused, train if fused else None, val if fused else None,
                     d_train if fused else None, plans if fused else None, X_train, X_val, oA, oB, output_length,
                     iter_start, max_iter, save_dir, check_every, verbose, save_plots, hook, runner=runner,
                     writer=writer)

    if fused:
        _eval_modes(model)
    restore_parameters(model, tr.best_model)
    if save_dir is not None and writer:
        torch.save(standalone_copy(model), os.path.join(save_dir, "final_best_model.bin"))
    if nsup > 0:
        final = model.validate_training(X_val, output_length, model.num_series, [], [], [], [], [])
        final_combo = final[-6]
    else:
        final_combo = model.validate_training(X_val, output_length, model.num_series)[-1]
    if verbose:
        print("FINAL BEST (STOPPING CRITERIA) LOSS == ", tr.best_loss, flush=True)
        print("FINAL BEST (STOPPING CRITERIA) EPOCH == ", tr.best_it, flush=True)
        print("FINAL VALIDATION COMBO LOSS == ", final_combo, flush=True)
    model.fit_history = tr.history()
    return final_combo


def save_checkpoint(model, save_dir, it, best_model, avg_forecasting_loss, avg_factor_loss,
                    avg_factor_cos_sim_penalty, avg_fw_l1_penalty, avg_fw_smoothing_penalty, avg_adj_penalty,
                    avg_dagness_reg_loss, avg_dagness_lag_loss, avg_dagness_node_loss, avg_combo_loss, best_loss,
                    best_it, f1score_histories, f1score_OffDiag_histories, roc_auc_histories,
                    roc_auc_OffDiag_histories, gc_factor_l1_loss_histories, gc_factor_cosine_sim_histories,
                    gc_factorUnsupervised_cosine_sim_histories, deltacon0_histories,
                    deltacon0_with_directed_degrees_histories, deltaffinity_histories, path_length_mse_histories,
                    GC=None, X_vis=None, cm_train=None, cm_val=None, save_plots=False, optimizers=None, **unused):
    """Writes the two files the reference's evaluation scripts and resume logic read
    (...withStateSmoothing.py:936-990).  Plots (general_utils/plotting.py) are out of scope.
    The model is saved as a standalone copy (its own parameter storage, not the pack's).
    With `optimizers` (fit passes its two Adams) a third file, optimizer_state.pt, holds their
    state: the reference does not checkpoint it (redcliff_s_cmlp.py:245), so a resumed
    reference fit restarts Adam, and so does resume_training_from_checkpoint here by default;
    with load_optimizer_state=True it loads the file, which makes a resumed fit continue
    exactly (tests/test_gpu_checkpoint.py)."""
    os.makedirs(save_dir, exist_ok=True)
    torch.save(standalone_copy(best_model), os.path.join(save_dir, "final_best_model.bin"))
    if optimizers is not None:
        torch.save(dict(zip(("A", "B"), (_compact_optimizer_state(o) for o in optimizers))),
                   os.path.join(save_dir, "optimizer_state.pt"))
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
