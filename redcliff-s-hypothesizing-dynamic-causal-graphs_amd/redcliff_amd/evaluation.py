"""Evaluation GC -> F1 pipeline: what the reference's evaluation
scripts do with a trained REDCLIFF-S model's causal-graph estimates.

Restated from
  * general_utils/metrics.py  compute_optimal_f1 :11-31, compute_f1 :34-41,
    compute_true_PosNeg_and_false_PosNeg_rates / sensitivity / specificity / LR+ / LR-
    :43-71, deltacon0 (with the ``make_graphs_undirected`` option) :162-189,
    solve_linear_sum_assignment_between_graph_options :274-301, compute_mse :384-386;
  * general_utils/misc.py  sort_unsupervised_estimates :83-91;
  * evaluate/eval_utils.py  compute_OptimalF1_stats_betw_two_gc_graphs :656-678,
    compute_f1_stats_betw_two_gc_graphs :681-703, compute_key_stats_betw_two_gc_graphs
    :706-746, get_combined_gc_representations_across_factors :884-891,
    get_model_gc_estimates :908-950 (REDCLIFF branch), and the factor-level statistics
    loop of perform_system_level_estimation_evaluation_of_cv_model :1244-1420.

The reference scores one (p x p) graph at a time through sklearn
(``precision_recall_curve``, ``f1_score``, ``confusion_matrix``, ``roc_auc_score``).  A
grid search produces thousands of estimates, so here every score is computed for a
whole stack of graphs at once: one stable descending sort per graph row, cumulative
true-positive counts, and the precision / recall / F1 arithmetic in the same float64
operation order as sklearn + the reference, so optimal thresholds, thresholded graphs
and F1 values are bit-identical to the reference's (tests/test_evaluation.py, pinned to
tests/golden/eval_pipeline.npz produced by the reference functions themselves).
ROC-AUC is the trapezoid over all distinct thresholds (sklearn drops collinear points
first), equal to the reference's to ~1e-15.
"""
import copy

import numpy as np
from scipy.optimize import linear_sum_assignment

from . import metrics as M

DEFAULT_PRED_CUTOFFS = (0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9)


# ----------------------------------------------------------------------------------------
# batched binary-classification curves (one row per graph)
# ----------------------------------------------------------------------------------------
def _as_rows(scores, labels):
    s = np.asarray(scores, dtype=np.float64)
    y = np.asarray(labels)
    if s.ndim == 1:
        s, y = s[None], y[None]
    s = s.reshape(s.shape[0], -1)
    y = (y.reshape(y.shape[0], -1) == 1)          # sklearn: y_true == pos_label (1)
    if s.shape != y.shape:
        raise ValueError("scores %s and labels %s differ in shape" % (s.shape, y.shape))
    return s, y


def _curve_rows(s, y):
    """sklearn _binary_clf_curve for every row: scores sorted descending (stable
    mergesort of the ascending order, reversed), tps/fps at each position, and a mask of
    the positions that end a run of equal scores (the curve's thresholds)."""
    order = np.argsort(s, axis=1, kind="mergesort")[:, ::-1]
    ss = np.take_along_axis(s, order, axis=1)
    yy = np.take_along_axis(y, order, axis=1).astype(np.float64)
    tps = np.cumsum(yy, axis=1)
    fps = 1.0 + np.arange(s.shape[1], dtype=np.float64)[None, :] - tps
    end = np.ones(s.shape, dtype=bool)
    end[:, :-1] = np.diff(ss, axis=1) != 0
    return ss, tps, fps, end


def batched_optimal_f1(scores, labels):
    """compute_optimal_f1 (metrics.py:11-31) for N graphs at once.

    scores, labels: (N, M) (or (M,)); labels in {0, 1}.  Returns (thresholds (N,),
    f1 (N,)).  Among equal maxima the reference's argmax over the ascending-threshold
    curve picks the LOWEST threshold; so does this."""
    s, y = _as_rows(scores, labels)
    ss, tps, fps, end = _curve_rows(s, y)
    precision = tps / (tps + fps)
    P = tps[:, -1:]
    recall = np.where(P == 0, 1.0, tps / np.where(P == 0, 1.0, P))
    with np.errstate(divide="ignore", invalid="ignore"):
        f1 = (2.0 * precision * recall) / (precision + recall)
    f1 = np.where(np.isfinite(f1), f1, 0.0)
    f1 = np.where(end, f1, -np.inf)
    best = f1.max(axis=1)
    # last sorted position (= lowest threshold) among the maxima
    pos = s.shape[1] - 1 - np.argmax((f1 == best[:, None])[:, ::-1], axis=1)
    thr = ss[np.arange(s.shape[0]), pos]
    return thr, best


def batched_roc_auc(scores, labels):
    """roc_auc_score (binary) for N graphs at once: trapezoid of (fpr, tpr) over the
    distinct thresholds, starting at (0, 0).  Rows with a single class give NaN (the
    reference raises there and records None)."""
    s, y = _as_rows(scores, labels)
    ss, tps, fps, end = _curve_rows(s, y)
    out = np.full(s.shape[0], np.nan)
    for r in range(s.shape[0]):
        t, f = tps[r][end[r]], fps[r][end[r]]
        if t[-1] == 0 or f[-1] == 0:
            continue
        tpr = np.concatenate(([0.0], t / t[-1]))
        fpr = np.concatenate(([0.0], f / f[-1]))
        out[r] = float(np.trapezoid(tpr, fpr))
    return out


def batched_confusion(scores, labels, cutoff):
    """(tp, tn, fp, fn) int64 arrays for predictions ``score > cutoff`` (metrics.py:36,
    :45-46)."""
    s, y = _as_rows(scores, labels)
    pred = s > cutoff
    tp = np.sum(pred & y, axis=1)
    tn = np.sum(~pred & ~y, axis=1)
    fp = np.sum(pred & ~y, axis=1)
    fn = np.sum(~pred & y, axis=1)
    return tp, tn, fp, fn


def batched_f1_at_cutoff(scores, labels, cutoff):
    """sklearn f1_score(labels, score > cutoff) per row (metrics.py:34-41): 2tp/(2tp+fp+fn),
    0 when there is no positive prediction nor label."""
    tp, _, fp, fn = batched_confusion(scores, labels, cutoff)
    den = 2 * tp + fp + fn
    return np.where(den == 0, 0.0, (2.0 * tp) / np.where(den == 0, 1, den))


# ----------------------------------------------------------------------------------------
# reference per-graph API (same names, arguments and edge cases)
# ----------------------------------------------------------------------------------------
def compute_optimal_f1(labels, pred_logits):
    thr, f1 = batched_optimal_f1(np.asarray(pred_logits)[None], np.asarray(labels)[None])
    assert np.isfinite(f1[0])
    return thr[0], f1[0]


def compute_f1(labels, pred_logits, pred_cutoff):
    return float(batched_f1_at_cutoff(np.asarray(pred_logits)[None], np.asarray(labels)[None], pred_cutoff)[0])


def compute_true_PosNeg_and_false_PosNeg_rates(labels, preds, pred_cutoff=None):
    preds = np.asarray(preds, dtype=np.float64)
    if pred_cutoff is None:  # hard predictions: positive iff == 1 (confusion_matrix labels)
        preds, pred_cutoff = (preds == 1).astype(np.float64), 0.5
    tp, tn, fp, fn = batched_confusion(preds[None], np.asarray(labels)[None], pred_cutoff)
    return np.int64(tp[0]), np.int64(tn[0]), np.int64(fp[0]), np.int64(fn[0])


def compute_sensitivity(labels, preds, pred_cutoff=None):
    tp, _, _, fn = compute_true_PosNeg_and_false_PosNeg_rates(labels, preds, pred_cutoff)
    with np.errstate(divide="ignore", invalid="ignore"):
        return tp / (tp + fn)


def compute_specificity(labels, preds, pred_cutoff=None):
    _, tn, fp, _ = compute_true_PosNeg_and_false_PosNeg_rates(labels, preds, pred_cutoff)
    with np.errstate(divide="ignore", invalid="ignore"):
        return tn / (tn + fp)


def compute_positive_likelihood_ratio(labels, preds, pred_cutoff=None):
    sens = compute_sensitivity(labels, preds, pred_cutoff)
    spec = compute_specificity(labels, preds, pred_cutoff)
    with np.errstate(divide="ignore", invalid="ignore"):
        return sens / (1. - spec)


def compute_negative_likelihood_ratio(labels, preds, pred_cutoff=None):
    sens = compute_sensitivity(labels, preds, pred_cutoff)
    spec = compute_specificity(labels, preds, pred_cutoff)
    with np.errstate(divide="ignore", invalid="ignore"):
        return (1. - sens) / spec


def compute_mse(A, B):
    return ((A - B) ** 2).mean()


def deltacon0(A1, A2, eps, make_graphs_undirected=False):
    """metrics.py:162-189, including the in-place symmetrisation order of the
    ``make_graphs_undirected`` option (G[j,i] takes the max after G[i,j] was updated)."""
    G1, G2 = np.array(A1, copy=True), np.array(A2, copy=True)
    assert G1.shape == G2.shape and G1.ndim == 2 and G1.shape[0] == G1.shape[1]
    if make_graphs_undirected:
        for G in (G1, G2):
            up = np.triu(G, 1)
            lo = np.tril(G, -1)
            m = np.maximum(lo, up.T)
            G[:] = np.diag(np.diag(G)) + m + m.T
    return M.deltacon0(G1, G2, eps)


def _labels_int(true_A):
    try:
        return np.array([int(v) for v in np.asarray(true_A).flatten()])
    except (TypeError, ValueError):
        return None


def _edge_case(est_A, true_A, labels):
    """The guard chain shared by eval_utils.py:665-673 / :690-698 / :714-722; True when the
    reference returns an empty dict (after printing a warning)."""
    if not np.isfinite(np.sum(est_A)):
        return True
    if np.min(est_A) == np.max(est_A):
        return True
    if not np.isfinite(np.sum(true_A)):
        return True
    if np.min(labels) == np.max(labels):
        return True
    return False


def compute_OptimalF1_stats_betw_two_gc_graphs(est_A, true_A):
    labels = _labels_int(true_A)
    if _edge_case(est_A, true_A, labels):
        return dict()
    thr, f1 = compute_optimal_f1(labels, np.asarray(est_A).flatten())
    return {"f1": f1, "decision_threshold": thr}


def compute_f1_stats_betw_two_gc_graphs(est_A, true_A, pred_cutoffs=DEFAULT_PRED_CUTOFFS):
    labels = _labels_int(true_A)
    if _edge_case(est_A, true_A, labels):
        return dict()
    flat = np.asarray(est_A).flatten()
    return dict(("f1_pc" + str(pc), compute_f1(labels, flat, pc)) for pc in pred_cutoffs)


def compute_key_stats_betw_two_gc_graphs(est_A, true_A, dcon0_eps=0.1, max_mse_path_length=None,
                                         make_graphs_undirected_for_dcon0=False, pred_cutoffs=DEFAULT_PRED_CUTOFFS):
    labels = _labels_int(true_A)
    if _edge_case(est_A, true_A, labels):
        return dict()
    flat = np.asarray(est_A).flatten()
    auc = batched_roc_auc(flat[None], labels[None])[0]
    stats = {"roc_auc": None if not np.isfinite(auc) else auc}
    for pc in pred_cutoffs:
        stats["sensitivity_pc" + str(pc)] = compute_sensitivity(labels, flat, pred_cutoff=pc)
        stats["specificity_pc" + str(pc)] = compute_specificity(labels, flat, pred_cutoff=pc)
        stats["PLR_pc" + str(pc)] = compute_positive_likelihood_ratio(labels, flat, pred_cutoff=pc)
        stats["NLR_pc" + str(pc)] = compute_negative_likelihood_ratio(labels, flat, pred_cutoff=pc)
    return stats


# ----------------------------------------------------------------------------------------
# estimates, sorting and the system-level factor statistics
# ----------------------------------------------------------------------------------------
def get_combined_gc_representations_across_factors(estimated_gcs, true_gcs):
    combo_true = np.zeros(true_gcs[0].shape)
    for t in true_gcs:
        combo_true = combo_true + t
    combo_est = np.zeros(estimated_gcs[0].shape)
    for e in estimated_gcs:
        combo_est = combo_est + e
    return combo_est, combo_true


def get_model_gc_estimates(model, model_type, num_ests_required, X=None):
    """REDCLIFF branch of eval_utils.py:908-925: the primary-mode GC of the single sample
    in ``X`` (lagged, unthresholded), one (p, p, L') array per factor, replicated when the
    mode yields one graph."""
    if "REDCLIFF" not in model_type:
        raise NotImplementedError("only REDCLIFF models are part of this build (model_type=%r)" % model_type)
    by_sample = model.GC(model.primary_gc_est_mode, X=X, threshold=False, ignore_lag=False,
                         combine_wavelet_representations=True, rank_wavelets=False)
    assert len(by_sample) == 1
    ests = [x.detach().cpu().numpy() for x in by_sample[0]]
    if len(ests) < num_ests_required:
        assert len(ests) == 1
        ests = [copy.deepcopy(ests[0]) for _ in range(num_ests_required)]
    return ests


def solve_linear_sum_assignment_between_graph_options(graph_estimates, true_graphs, cost_criteria="CosineSimilarity",
                                                      inf_approximation=10000000000.):
    """metrics.py:274-301.  The cost IS the cosine similarity (minimised, as the reference
    does); non-finite costs become ``inf_approximation``."""
    if cost_criteria != "CosineSimilarity":
        raise NotImplementedError()
    cost = np.zeros((len(graph_estimates), len(true_graphs)))
    for w, g in enumerate(graph_estimates):
        for j, t in enumerate(true_graphs):
            cost[w, j] += M.compute_cosine_similarity(g, t)
    bad = ~np.isfinite(cost)
    cost[bad] = 0.
    return linear_sum_assignment(cost + inf_approximation * bad)


def sort_unsupervised_estimates(graph_estimates, true_graphs, cost_criteria="CosineSimilarity",
                                unsupervised_start_index=0, return_sorting_inds=False):
    """misc.py:83-91."""
    ests, trues = graph_estimates[unsupervised_start_index:], true_graphs[unsupervised_start_index:]
    est_inds, gt_inds = solve_linear_sum_assignment_between_graph_options(ests, trues, cost_criteria="CosineSimilarity")
    sorted_ests = [None for _ in range(len(trues))]
    for e, g in zip(est_inds, gt_inds):
        sorted_ests[g] = ests[e]
    unsorted = [ests[i] for i in range(len(ests)) if i not in est_inds]
    out = graph_estimates[:unsupervised_start_index] + sorted_ests + unsorted
    if return_sorting_inds:
        return out, est_inds, gt_inds
    return out


FACTOR_STATS = ("cos_sim", "mse", "dir_deltacon0", "undir_deltacon0", "deltacon0_wDD", "deltaffinity", "roc_auc")


def system_level_factor_stats(gc_factor_ests, true_gc_factors, eps=0.1, in_degree_coeff=1., out_degree_coeff=1.,
                              max_path_length=None, sort_unsupervised_ests=False, cost_criteria="CosineSimilarity",
                              unsupervised_start_index=0, average_estimated_graphs_together=False,
                              exclude_self_connections=False, evaluate_identity_baseline=False):
    """One model's factor-level statistics, as eval_utils.py:1244-1420 computes them for each
    trained fold: optional sorting of unsupervised estimates, identity baseline, removal of
    self-connections, normalisation by the maximum, optional averaging, lag sums, then per
    factor the cosine similarity, MSE, directed / undirected deltacon0, deltacon0 with
    directed degrees, deltaffinity and ROC-AUC -- each also against the transposed
    estimate ("T_" keys).  Returns {stat: per-factor list, stat + "_avg", stat + "_std"}
    (averages divide by the number of true factors, as the reference does)."""
    ests = list(gc_factor_ests)
    if sort_unsupervised_ests:
        ests = sort_unsupervised_estimates(ests, true_gc_factors, cost_criteria=cost_criteria,
                                           unsupervised_start_index=unsupervised_start_index)
    if evaluate_identity_baseline:
        ests = [np.expand_dims(np.eye(e.shape[0]), 2) + (0. * e) for e in ests]
    if exclude_self_connections:
        ests = [(1. - np.expand_dims(np.eye(e.shape[0]), 2)) * e for e in ests]
    norm = [e / np.max(e) for e in ests]
    if evaluate_identity_baseline:
        norm = [e for e in ests]
    if average_estimated_graphs_together and len(norm) > len(true_gc_factors):
        assert len(true_gc_factors) == 1
        avg = np.zeros(norm[0].shape)
        for e in norm:
            avg = avg + e
        norm = [(1. / len(norm)) * avg]

    out = dict((("T_" if t else "") + k, []) for k in FACTOR_STATS for t in (False, True))
    for true_gc, gc_est in zip(true_gc_factors, norm):
        assert true_gc.ndim == 3
        true_gc = true_gc.sum(axis=2)
        if gc_est.ndim == 3:
            gc_est = gc_est.sum(axis=2)
        assert np.isfinite(true_gc.sum()) and np.isfinite(gc_est.sum())
        labels = [int(v) for v in (1. * (true_gc > 0.)).flatten()]
        for T, est in (("", gc_est), ("T_", gc_est.T)):
            out[T + "cos_sim"].append(M.compute_cosine_similarity(true_gc, est))
            out[T + "mse"].append(compute_mse(true_gc, est))
            out[T + "dir_deltacon0"].append(deltacon0(true_gc, est, eps, make_graphs_undirected=False))
            out[T + "undir_deltacon0"].append(deltacon0(true_gc, est, eps, make_graphs_undirected=True))
            out[T + "deltacon0_wDD"].append(M.deltacon0_with_directed_degrees(
                true_gc, est, eps, in_degree_coeff=in_degree_coeff, out_degree_coeff=out_degree_coeff))
            out[T + "deltaffinity"].append(M.deltaffinity(true_gc, est, eps, max_path_length=max_path_length))
            auc = batched_roc_auc(est.flatten()[None], np.asarray(labels)[None])[0]
            if not np.isfinite(auc):
                raise ValueError("roc_auc_score: only one class present in the true graph")
            out[T + "roc_auc"].append(auc)
    n = len(true_gc_factors)
    for k in list(out):
        vals = out[k]
        out[k + "_avg"] = sum(vals) / n if vals else 0.
        out[k + "_std"] = float(np.std(vals))
    return out


def batched_graph_f1(est_stack, true_stack, normalize=True, lag_sum=True, exclude_self_connections=False):
    """Optimal-F1 scoring of many estimates at once (a grid search's worth): est_stack
    (N, p, p[, L]) against true_stack (N, p, p[, L']) -- each estimate normalised by its
    maximum and summed over lags as in the system-level pipeline, labels = true > 0.
    Returns dict(f1 (N,), threshold (N,), roc_auc (N,), graphs (N, p, p) int -- the
    estimates thresholded at their optimal decision threshold, ``score >= threshold``
    (sklearn's precision_recall_curve convention))."""
    E = np.asarray(est_stack, dtype=np.float64)
    Tg = np.asarray(true_stack, dtype=np.float64)
    if exclude_self_connections:
        eye = np.eye(E.shape[1])
        E = E * (1. - (eye[..., None] if E.ndim == 4 else eye))
    if normalize:
        E = E / E.reshape(E.shape[0], -1).max(axis=1).reshape((-1,) + (1,) * (E.ndim - 1))
    if lag_sum and E.ndim == 4:
        E = E.sum(axis=3)
    if Tg.ndim == 4:
        Tg = Tg.sum(axis=3)
    labels = (Tg > 0.).astype(np.int64)
    thr, f1 = batched_optimal_f1(E.reshape(E.shape[0], -1), labels.reshape(E.shape[0], -1))
    auc = batched_roc_auc(E.reshape(E.shape[0], -1), labels.reshape(E.shape[0], -1))
    graphs = (E >= thr[:, None, None]).astype(np.int64)
    return dict(f1=f1, threshold=thr, roc_auc=auc, graphs=graphs)
