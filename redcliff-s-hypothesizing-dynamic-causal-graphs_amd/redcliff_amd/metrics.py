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


def _approx_affinity(A, eps, kmax):
    """metrics.py:142-160: S = I, then S = S + (1.*(eps**k)) * A^k in order (float64 S, the
    terms in A's dtype)."""
    S = np.eye(A.shape[0])
    for k, Ak in enumerate(_path_powers(A, kmax), start=1):
        S = S + (1. * (eps ** k) * Ak)
    return S


def deltaffinity(A1, A2, eps, max_path_length=None):
    n = A1.shape[0]
    kmax = n - 1 if max_path_length is None else max_path_length
    return 1. / (1. + _matsusita(_approx_affinity(A1, eps, kmax), _approx_affinity(A2, eps, kmax)))


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
                e = np.array(est)  # the estimate's own dtype (float32), as the reference
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
            e = np.array(est)
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


# ---------------------------------------------------------------------------------------------
# GPU path (rc_metrics.hip, redcliff_gc_progress): the same per-(sample, graph) values computed
# on the device in one launch, then accumulated over samples on the host exactly as the
# reference's trackers accumulate them (python-float running sums, division by the sample
# count, the length-mismatch rules of model_utils.py:63-84 / :136-158).

def _truth_arrays(GC, G):
    on = np.stack([_prep_true(np.asarray(GC[g], dtype=np.float64), False) for g in range(G)])
    off = np.stack([_prep_true(np.asarray(GC[g], dtype=np.float64), True) for g in range(G)])
    return np.ascontiguousarray(np.stack([on, off]), dtype=np.float64)


_TRUTH_CACHE = []  # [(GC list object, its arrays' ids, G, p, eps, device, truth, eps_pow)]: a fit's constants


def _device_truth(GC, G, p, eps, dev):
    """The normalised true graphs and eps powers on the device, uploaded once per fit (same GC
    list object and arrays) instead of once per epoch."""
    ids = tuple(id(g) for g in GC)
    for ent in _TRUTH_CACHE:
        if ent[0] is GC and ent[1] == ids and ent[2:6] == (G, p, eps, dev):
            return ent[6], ent[7]
    truth = torch.from_numpy(_truth_arrays(GC, G)).to(dev)
    eps_pow = torch.tensor([eps ** k for k in range(p)], dtype=torch.float64, device=dev)
    _TRUTH_CACHE.insert(0, (GC, ids, G, p, eps, dev, truth, eps_pow))
    del _TRUTH_CACHE[16:]
    return truth, eps_pow


def _used_here(truth, eps_pow, dev):
    """A cached truth table may be read on another stream than the one it was allocated on (packs
    fitted concurrently by fit_packs, one stream each, sharing one true-graph list): tell the
    caching allocator, so evicting the entry never frees memory a pending launch still reads."""
    s = torch.cuda.current_stream(dev)
    truth.record_stream(s)
    eps_pow.record_stream(s)


def gc_progress_values(GC, est, eps=0.1, in_degree_coeff=1., out_degree_coeff=1., host=True):
    """est: float32 CUDA tensor (S, nE, p, p, Lt) of GC estimates; GC: true graphs (p, p, lags).
    Returns float64 (S, G, 6 + p), G = min(nE, len(GC)): f1, roc_auc, f1 / roc_auc without
    self-connections, deltacon0, deltacon0 with directed degrees, deltaffinity, path-length MSE
    k = 1..p-1 -- the per-sample values the reference trackers sum."""
    import ctypes
    from . import _native as nat
    S, nE, p, p2, Lt = est.shape
    assert p == p2
    G = min(nE, len(GC))
    dev = est.device
    est = est.to(torch.float32).contiguous()
    truth, eps_pow = _device_truth(GC, G, p, eps, dev)
    _used_here(truth, eps_pow, dev)
    out = torch.empty(S, G, 6 + p, dtype=torch.float64, device=dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    nat.check(nat.lib().redcliff_gc_progress(S, nE, G, p, Lt, est.data_ptr(), truth.data_ptr(), eps_pow.data_ptr(),
                                              float(in_degree_coeff), float(out_degree_coeff), out.data_ptr(), stream),
              "gc_progress")
    return out.cpu().numpy() if host else out


def gc_progress_values_grouped(GCs, est, spt, eps=0.1, in_degree_coeff=1., out_degree_coeff=1., host=True):
    """gc_progress_values with one list of true graphs per group of `spt` consecutive samples
    (GCs[i] scores samples i*spt .. i*spt+spt-1): the per-replica true graphs of a packed grid
    whose replicas fit different data sets.  Every GCs[i] holds the same number of graphs."""
    import ctypes
    from . import _native as nat
    S, nE, p, p2, Lt = est.shape
    assert p == p2 and S == spt * len(GCs), (S, spt, len(GCs))
    G = min([nE] + [len(g) for g in GCs])
    if any(len(g) != len(GCs[0]) for g in GCs):
        raise ValueError("per-replica true graphs must have one length")
    dev = est.device
    est = est.to(torch.float32).contiguous()
    ids = tuple(id(x) for g in GCs for x in g)
    hit = None
    for ent in _TRUTH_CACHE:
        if ent[0] is GCs and ent[1] == ids and ent[2:6] == (G, p, eps, dev):
            hit = ent
            break
    if hit is None:
        truth = torch.from_numpy(np.ascontiguousarray(np.stack([_truth_arrays(g, G) for g in GCs]))).to(dev)
        eps_pow = torch.tensor([eps ** k for k in range(p)], dtype=torch.float64, device=dev)
        hit = (GCs, ids, G, p, eps, dev, truth, eps_pow)
        _TRUTH_CACHE.insert(0, hit)
        del _TRUTH_CACHE[16:]
    truth, eps_pow = hit[6], hit[7]
    _used_here(truth, eps_pow, dev)
    out = torch.empty(S, G, 6 + p, dtype=torch.float64, device=dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    nat.check(nat.lib().redcliff_gc_progress_grouped(S, spt, nE, G, p, Lt, est.data_ptr(), truth.data_ptr(),
                                                      eps_pow.data_ptr(), float(in_degree_coeff),
                                                      float(out_degree_coeff), out.data_ptr(), stream),
              "gc_progress_grouped")
    return out.cpu().numpy() if host else out


def _running(vals):
    """Per-graph running sums over samples in sample order (python floats), and the count."""
    run = None
    for s in range(vals.shape[0]):
        row = [float(v) for v in vals[s]]
        run = row if run is None else [a + b for a, b in zip(run, row)]
    return (run or []), float(vals.shape[0])


def track_roc_stats_from_values(vals, f1_hist, roc_hist, remove_self_connections=False):
    """track_roc_stats with the device values (thresholds other than 0.0 are not on the device path)."""
    col = 2 if remove_self_connections else 0
    for thresh in f1_hist.keys():
        if thresh != 0.0:
            raise ValueError("device GC-progress metrics cover the fit's threshold 0.0 only")
        f1_run, n = _running(vals[:, :, col])
        roc_run, _ = _running(vals[:, :, col + 1])
        if len(f1_hist[thresh]) != len(f1_run):
            if len(f1_run) == 1 and len(f1_hist[thresh]) > 1:
                for i in range(len(f1_hist[thresh])):
                    f1_hist[thresh][i].append(f1_run[0] / n)
                    roc_hist[thresh][i].append(roc_run[0] / n)
                continue
            assert len(f1_hist[thresh]) < len(f1_run)
        for i in range(len(f1_hist[thresh])):
            f1_hist[thresh][i].append(f1_run[i] / n)
            roc_hist[thresh][i].append(roc_run[i] / n)
    return f1_hist, roc_hist


def track_deltacon_stats_from_values(vals, num_chans, dc_hist, dcdd_hist, daff_hist, plm_hist):
    """track_deltacon_stats with the device values."""
    dc, n = _running(vals[:, :, 4])
    dcdd, _ = _running(vals[:, :, 5])
    daff, _ = _running(vals[:, :, 6])
    p = vals.shape[2] - 6
    plm = {pl: _running(vals[:, :, 6 + pl])[0] for pl in range(1, min(num_chans, p))}
    if len(dc_hist) != len(dc):
        if len(dc) == 1 and len(dc_hist) > 1:
            for i in range(len(dc_hist)):
                dc_hist[i].append(dc[0] / n)
                dcdd_hist[i].append(dcdd[0] / n)
                daff_hist[i].append(daff[0] / n)
            return dc_hist, dcdd_hist, daff_hist, plm_hist
        assert len(dc_hist) < len(dc)
        for i in range(len(dc_hist)):
            dc_hist[i].append(dc[i] / n)
            dcdd_hist[i].append(dcdd[i] / n)
            daff_hist[i].append(daff[i] / n)
        return dc_hist, dcdd_hist, daff_hist, plm_hist
    for i in range(len(dc_hist)):
        dc_hist[i].append(dc[i] / n)
        dcdd_hist[i].append(dcdd[i] / n)
        daff_hist[i].append(daff[i] / n)
        for pl in plm.keys():
            plm_hist[pl][i].append(plm[pl][i] / n)
    return dc_hist, dcdd_hist, daff_hist, plm_hist


def track_cosine_stats_batched(est, hist, label_offset=0):
    """track_cosine_stats on a stacked (S, K, ...) array in one vectorised pass (float64, as
    compute_cosine_similarity above)."""
    a = np.asarray(est, dtype=np.float64)
    S, K = a.shape[0], a.shape[1]
    if K < 2 or S == 0:
        return hist
    flat = a.reshape(S, K, -1)
    flat = flat / flat.max(axis=2, keepdims=True)
    with np.errstate(invalid="ignore"):
        nrm = np.linalg.norm(flat, axis=2)
    nrm = np.where(np.isfinite(nrm), nrm, -1.)
    nrm = np.maximum(nrm, 1e-8)
    dots = np.einsum("ski,sli->skl", flat, flat)
    cur = {}
    for i1 in range(K):
        for i2 in range(i1 + 1, K):
            v = dots[:, i1, i2] / (nrm[:, i1] * nrm[:, i2])
            tot = 0.
            for x in v:
                tot += float(x)
            cur["%dand%d" % (i1 + label_offset, i2 + label_offset)] = tot
    for key in cur:
        hist[key].append(cur[key] / float(S))
    return hist


# ---------------------------------------------------------------------------------------------
# Tracker statistics of fit() (model_utils.py:163-209): the per-(sample, factor) L1 values of the
# lagged estimates and the normalised dot products of the lag-free estimates, computed on the
# device (redcliff_gc_track_stats) so only [S][K] / [Sn][K][K] values cross to the host; the
# python-float bookkeeping (running sums over samples, pairs, history appends) is
# fit_loop.gc_progress_many.  track_values_host is the same quantities in the reference's numpy
# order (test oracle for the device values).

def gc_track_values(est, nolag, host=True):
    """est (..., S, K, p, p, Ls) and nolag (..., Sn, K, p, p, 1) float32 CUDA tensors ->
    (l1 (..., S, K), nrm (..., Sn, K), dots (..., Sn, K, K)) float64 numpy (dots: upper triangle).
    host=False: (l1, dots) still on the device (finish with track_values_finish)."""
    import ctypes
    from . import _native as nat
    dev = est.device
    lead = est.shape[:-5]
    S, K = est.shape[-5], est.shape[-4]
    Sn = nolag.shape[-5]
    est = est.to(torch.float32).contiguous()
    nolag = nolag.to(torch.float32).contiguous()
    nrow = int(np.prod(lead, dtype=np.int64)) * S * K
    nsamp = int(np.prod(lead, dtype=np.int64)) * Sn
    l1 = torch.zeros(max(nrow, 1), dtype=torch.float64, device=dev)
    dots = torch.zeros(max(nsamp, 1), K, K, dtype=torch.float64, device=dev)
    row = int(np.prod(est.shape[-3:]))
    rown = int(np.prod(nolag.shape[-3:]))
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    nat.check(nat.lib().redcliff_gc_track_stats(nrow, row, est.data_ptr(), l1.data_ptr(), nsamp, K, rown,
                                                nolag.data_ptr(), dots.data_ptr(), stream), "gc_track_stats")
    l1 = l1[:nrow].view(tuple(lead) + (S, K))
    dots = dots[:nsamp].view(tuple(lead) + (Sn, K, K))
    if not host:
        return l1, dots
    return track_values_finish(l1.cpu().numpy(), dots.cpu().numpy())


def track_values_finish(l1, dots):
    """(l1, nrm, dots) host arrays from the device statistics (nrm = sqrt of the diagonal)."""
    return l1, np.sqrt(np.diagonal(dots, axis1=-2, axis2=-1)), dots


class _PendingFetch:
    """fetch_async's handle: the packed values are on their way into pinned host memory."""

    def __init__(self, tensors):
        flat = torch.cat([t.reshape(-1).to(torch.float64) for t in tensors])
        self.host = torch.empty(flat.shape, dtype=torch.float64, pin_memory=True)
        self.host.copy_(flat, non_blocking=True)
        self.ev = torch.cuda.Event()
        self.ev.record()
        self.meta = [(tuple(t.shape), t.dtype, t.numel()) for t in tensors]

    def wait(self):
        self.ev.synchronize()
        flat = self.host.numpy()
        out, o = [], 0
        for shape, dt, n in self.meta:
            a = flat[o:o + n].reshape(shape)
            out.append(a.copy() if dt == torch.float64 else a.astype(np.int64))
            o += n
        return out


def fetch_async(tensors):
    """fetch() without waiting: the copy is enqueued on the current stream (later launches may
    follow it); .wait() blocks until the copy itself has landed and returns the arrays."""
    return _PendingFetch(tensors)


def fetch(tensors):
    """ONE device -> host copy of several small tensors (float64 / integer counts, exact as
    float64): numpy arrays of their shapes (integers come back as int64)."""
    flat = torch.cat([t.reshape(-1).to(torch.float64) for t in tensors]).cpu().numpy()
    out, o = [], 0
    for t in tensors:
        a = flat[o:o + t.numel()].reshape(tuple(t.shape))
        out.append(a if t.dtype == torch.float64 else a.astype(np.int64))
        o += t.numel()
    return out


def track_values_host(est, nolag):
    """gc_track_values on host arrays, in the per-fit trackers' numpy order (track_l1_stats:
    np.sum(np.abs(e / np.max(e))) per estimate; track_cosine_stats_batched: np.linalg.norm and
    einsum of the max-normalised rows)."""
    e = np.asarray(est, dtype=np.float64)
    lead = e.shape[:-3]
    mx = e.max(axis=(-3, -2, -1), keepdims=True)
    l1 = np.abs(e / mx).reshape(lead + (-1,)).sum(axis=-1)
    a = np.asarray(nolag, dtype=np.float64)
    flat = a.reshape(a.shape[:-3] + (-1,))
    flat = flat / flat.max(axis=-1, keepdims=True)
    with np.errstate(invalid="ignore"):
        nrm = np.linalg.norm(flat, axis=-1)
    dots = np.einsum("...ki,...li->...kl", flat, flat)
    return l1, nrm, dots
