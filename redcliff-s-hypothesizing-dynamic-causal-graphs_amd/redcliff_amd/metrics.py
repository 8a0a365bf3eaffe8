"""Host-side graph metrics used by REDCLIFF-S ``fit`` for per-epoch GC-progress tracking.

Restated from general_utils/metrics.py (compute_cosine_similarity :321-339,
get_f1_score :396-430, deltacon0 :160-187, deltacon0_with_directed_degrees :189-216,
deltaffinity :218-234, path_length_mse :236-252) and the tracking helpers of
general_utils/model_utils.py:18-209.  They run once per epoch on <= 40 small (p x p)
matrices copied to the host, exactly as in the reference.
"""
import numpy as np
import torch
from sklearn.metrics import roc_auc_score


def compute_cosine_similarity(A, B, epsilon=1e-8):
    a = np.asarray(A, dtype=np.float64).ravel()
    b = np.asarray(B, dtype=np.float64).ravel()
    na, nb = np.linalg.norm(a), np.linalg.norm(b)
    na = na if np.isfinite(na) else -1.
    nb = nb if np.isfinite(nb) else -1.
    return np.dot(a, b) / (max(na, epsilon) * max(nb, epsilon))


def get_f1_score(A_hat, A):
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


def _affinity(D, A, eps):
    n = A.shape[0]
    return np.linalg.inv(np.eye(n) + (eps ** 2.) * D - eps * A)


def _matsusita(S1, S2):
    return np.sqrt(np.sum((np.sqrt(S1) - np.sqrt(S2)) ** 2.))


def deltacon0(A1, A2, eps):
    D1, D2 = np.diag(np.sum(A1, axis=0)), np.diag(np.sum(A2, axis=0))
    return 1. / (1. + _matsusita(_affinity(D1, A1, eps), _affinity(D2, A2, eps)))


def deltacon0_with_directed_degrees(A1, A2, eps, in_degree_coeff=1., out_degree_coeff=1.):
    d_in = _matsusita(_affinity(np.diag(np.sum(A1, axis=0)), A1, eps), _affinity(np.diag(np.sum(A2, axis=0)), A2, eps))
    d_out = _matsusita(_affinity(np.diag(np.sum(A1, axis=1)), A1, eps), _affinity(np.diag(np.sum(A2, axis=1)), A2, eps))
    return 1. / (1. + (in_degree_coeff * d_in + out_degree_coeff * d_out) / 2.)


def _path_powers(A, kmax):
    out, Ak = [], A
    for k in range(1, kmax + 1):
        if k > 1:
            Ak = np.dot(Ak, A)
        out.append(Ak)
    return out


def deltaffinity(A1, A2, eps, max_path_length=None):
    n = A1.shape[0]
    kmax = n - 1 if max_path_length is None else max_path_length
    S1 = np.eye(n) + sum((eps ** k) * Ak for k, Ak in enumerate(_path_powers(A1, kmax), start=1))
    S2 = np.eye(n) + sum((eps ** k) * Ak for k, Ak in enumerate(_path_powers(A2, kmax), start=1))
    return 1. / (1. + _matsusita(S1, S2))


def path_length_mse(A1, A2, max_path_length=None):
    kmax = A1.shape[0] - 1 if max_path_length is None else max_path_length
    mses = [((a - b) ** 2.).mean() for a, b in zip(_path_powers(A1, kmax), _path_powers(A2, kmax))]
    return sum(mses), mses


def _prep_true(G, remove_self):
    g = np.sum(G, axis=2)
    if remove_self:
        np.fill_diagonal(g, 0.)
    if np.max(g) != 0.:
        g = g / np.max(g)
    return g


def track_roc_stats(GC, CURR_GC_EST, f1_hist, roc_hist, remove_self_connections=False):
    """general_utils/model_utils.py:18-86"""
    for thresh in f1_hist.keys():
        n_samp, f1s, rocs = 0., [], []
        for s, ests in enumerate(CURR_GC_EST):
            for i, est in enumerate(ests[:len(GC)]):
                true = _prep_true(GC[i], remove_self_connections)
                e = np.asarray(est, dtype=np.float64)
                if e.ndim == 3:
                    e = np.sum(e, axis=2)
                if remove_self_connections:
                    e = e.copy()
                    np.fill_diagonal(e, 0.)
                if np.max(e) != 0.:
                    e = e / np.max(e)
                e = e * (e > thresh)
                labels = [int(v) for v in true.flatten()]
                f1 = get_f1_score(e, true)
                roc = 0.5 if np.sum(labels) == 0 else roc_auc_score(labels, e.flatten())
                if s == 0:
                    f1s.append(f1)
                    rocs.append(roc)
                else:
                    f1s[i] += f1
                    rocs[i] += roc
            n_samp += 1.
        hist_len = len(f1_hist[thresh])
        if hist_len != len(f1s) and len(f1s) == 1 and hist_len > 1:
            for i in range(hist_len):
                f1_hist[thresh][i].append(f1s[0] / n_samp)
                roc_hist[thresh][i].append(rocs[0] / n_samp)
        else:
            for i in range(hist_len):
                f1_hist[thresh][i].append(f1s[i] / n_samp)
                roc_hist[thresh][i].append(rocs[i] / n_samp)
    return f1_hist, roc_hist


def track_deltacon_stats(GC, CURR_GC_EST, num_chans, dc_hist, dcdd_hist, daff_hist, plm_hist, eps=0.1,
                         in_degree_coeff=1., out_degree_coeff=1.):
    """general_utils/model_utils.py:89-160 (remove_self_connections=False as called by fit)."""
    n_samp = 0.
    dc, dcdd, daff, plm = [], [], [], {}
    for s, ests in enumerate(CURR_GC_EST):
        for i, est in enumerate(ests[:len(GC)]):
            true = _prep_true(GC[i], False)
            e = np.asarray(est, dtype=np.float64)
            if e.ndim == 3:
                e = np.sum(e, axis=2)
            if np.max(np.sum(GC[i], axis=2)) != 0.:
                e = e / np.max(e)
            _, mses = path_length_mse(true, e)
            vals = (deltacon0(true, e, eps), deltacon0_with_directed_degrees(true, e, eps, in_degree_coeff, out_degree_coeff),
                    deltaffinity(true, e, eps))
            if s == 0:
                dc.append(vals[0])
                dcdd.append(vals[1])
                daff.append(vals[2])
                for pl, mse in zip(range(1, num_chans), mses):
                    plm.setdefault(pl, [0. for _ in range(len(ests))])
                    plm[pl][i] += mse
            else:
                dc[i] += vals[0]
                dcdd[i] += vals[1]
                daff[i] += vals[2]
                for pl, mse in zip(range(1, num_chans), mses):
                    plm[pl][i] += mse
        n_samp += 1.
    if len(dc_hist) != len(dc) and len(dc) == 1 and len(dc_hist) > 1:
        for i in range(len(dc_hist)):
            dc_hist[i].append(dc[0] / n_samp)
            dcdd_hist[i].append(dcdd[0] / n_samp)
            daff_hist[i].append(daff[0] / n_samp)
    else:
        for i in range(len(dc_hist)):
            dc_hist[i].append(dc[i] / n_samp)
            dcdd_hist[i].append(dcdd[i] / n_samp)
            daff_hist[i].append(daff[i] / n_samp)
            if len(dc_hist) == len(dc):
                for pl in plm.keys():
                    plm_hist[pl][i].append(plm[pl][i] / n_samp)
    return dc_hist, dcdd_hist, daff_hist, plm_hist


def track_l1_stats(CURR_GC_EST, l1_hist):
    """general_utils/model_utils.py:163-186"""
    run, n_samp = [], 0.
    for s, ests in enumerate(CURR_GC_EST):
        for k, est in enumerate(ests):
            e = np.asarray(est, dtype=np.float64)
            v = float(np.sum(np.abs(e / np.max(e))))
            if s == 0:
                run.append(v)
            else:
                run[k] += v
        n_samp += 1.
    run = [x / n_samp for x in run]
    for i in range(len(l1_hist)):
        l1_hist[i].append(run[i])
    return sum(run), l1_hist


def track_cosine_stats(CURR_GC_EST, hist, label_offset=0):
    """general_utils/model_utils.py:189-209"""
    cur, n_samp = {}, 0.
    for s, ests in enumerate(CURR_GC_EST):
        for i1, g1 in enumerate(ests):
            for i2, g2 in enumerate(ests):
                if i1 < i2:
                    a = np.asarray(g1, dtype=np.float64)
                    b = np.asarray(g2, dtype=np.float64)
                    v = compute_cosine_similarity(a / np.max(a), b / np.max(b))
                    key = "%dand%d" % (i1 + label_offset, i2 + label_offset)
                    cur[key] = v if s == 0 else cur[key] + v
        n_samp += 1.
    for key in cur:
        hist[key].append(cur[key] / n_samp)
    return hist
