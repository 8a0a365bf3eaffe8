"""Data side of the fitting path: the synthetic sVAR
generator and the normalised window set that feeds ``fit`` with device-resident batches.

* ``generate_synthetic_data`` restates data/data_utils.py:47-240
  (multivariate_relational_nvar_sinusoid_with_gaussian_innovations :47-86,
  sample_signal_from_system_state :89-128, sample_and_apply_linearly_interpolated_weights
  :131-137, generate_synthetic_data :140-240).  The reference steps one recording, one
  system state, one time step and one (receiver, sender, lag) edge at a time in Python
  (~17 s per 320 recordings).  Here every (recording, state) chain advances together:
  one array update per (sender, lag) per time step, the random numbers drawn from the
  same legacy ``RandomState`` stream in the reference's order (initial condition,
  innovations, interpolation weights per state, then the additive noise), and the float64
  arithmetic kept in the reference's order (per-receiver accumulation over senders, the
  self-edge term added at the receiver's own position), so with the same seed the
  recordings and labels are bit-identical to the reference's
  (tests/test_data.py against tests/golden/svar_data.npz).
* ``NormalizedWindowSet`` restates data/synthetic_datasets.py:18-160
  (NormalizedSyntheticWVARDataset): per-channel mean / standard deviation over every
  accepted recording and time step (sequential float64 sums, as the reference
  accumulates them file by file), NaN recordings skipped, one ``random.Random(seed)``
  shuffle, the grid-search quarter, and ``(x - mean) / std`` with x cast to float32
  first.  Instead of unpickling a subset file per ``__getitem__`` (the reference's loader
  reaches ~1.6 k samples/s), the normalised windows are materialised once and moved to
  HBM; ``batches`` then yields the DataLoader's batch sequence as views.

* ``NormalizedRecordingDirectory`` reads the reference's subset-pickle directories:
  ``kind="dream4"`` restates data/dream4_datasets.py:18-157 (NormalizedDREAM4Dataset: files
  named ``subset_*``, no grid-search cut) and ``kind="lfp"`` restates
  data/local_field_potential_datasets.py:18-187 (NormalizedLocalFieldPotentialDataset: files
  named ``*_subset*``, optional region averaging :118-132 applied before the statistics and
  to every item, the grid-search tenth :109-112); ``kind="synthetic"`` is
  NormalizedSyntheticWVARDataset's file filter.  Each file is unpickled once (the reference
  re-opens a file per sample in the statistics pass and per item), the statistics keep the
  reference's operation order on the arrays as stored, and the same shuffle / cut / item
  arithmetic applies; ``*_train_test_split`` mirror the loaders' ``train`` / ``validation``
  split (:168-189 / :198-219).

Per-edge activations are integer codes (``ACT_*``) instead of lambdas; the curation
script's two patterns are identity and ``[min(x, 0), max(x, 0)]`` per lag
(data/currate_sVARwInnovativeContinuousGaussianNoise_data_etNL.py:272-275).
"""
import os
import pickle
import random
import shutil

import numpy as np
import torch

ACT_NONE, ACT_IDENTITY, ACT_MIN0, ACT_MAX0 = 0, 1, 2, 3


def _act(code, x):
    """Apply per-(chain, receiver) activation codes to x (same shape as code)."""
    out = x
    out = np.where(code == ACT_MIN0, np.minimum(x, 0.0), out)
    out = np.where(code == ACT_MAX0, np.maximum(x, 0.0), out)
    return out


def _chain_step(h1, h2, A, codes, cos2, amp, noise, num_lags):
    """One reference time step for every chain.

    h1, h2: (C, D) the last and second-to-last states; A: (C, D, D, L) the chains'
    lagged adjacency (receiver, sender, lag); codes: (C, D, D, L) activation codes or
    None; cos2: (D,) 2*cos(2*pi*f); amp: (D,); noise: (C, D) the drawn innovations
    (mu + var * gauss).  Mirrors data_utils.py:69-85 term by term."""
    C, D = h1.shape
    x = np.zeros((C, D))
    hist = (h1, h2)
    rows = np.arange(D)
    for j in range(D):
        off = rows != j
        for l in range(num_lags):
            c = A[:, :, j, l] * hist[l][:, j:j + 1]
            if codes is not None:
                c = _act(codes[:, :, j, l], c)
            x = np.where(off[None, :], x + c, x)
        lag1 = A[:, j, j, 0] * (cos2[j] * h1[:, j])
        if codes is not None:
            lag1 = _act(codes[:, j, j, 0], lag1)
        lag2 = 0.
        if num_lags > 1:
            lag2 = A[:, j, j, 1] * (-1 * h2[:, j])
            if codes is not None:
                lag2 = _act(codes[:, j, j, 1], lag2)
        x[:, j] = x[:, j] + (lag1 + lag2 + amp[j] * noise[:, j])
    return x


def generate_synthetic_data(num_samples, recording_length, label_type, burnin_period, D, num_possible_states,
                            num_labeled_states, n_lags, lagged_adj_graphs, base_freqs, noise_mu, noise_var,
                            innovation_amp_coeffs, noise_amp_coeffs, noise_type="white", activation_codes=None,
                            rng=None):
    """data_utils.generate_synthetic_data without plotting.

    lagged_adj_graphs: (S, D, D, L) per system state; activation_codes: None or
    (S, D, D, L) ints (ACT_*); base_freqs / noise_mu / noise_var / innovation_amp_coeffs:
    (D, 1) arrays as in the reference; rng: a ``numpy.random.RandomState`` (default: the
    global legacy generator, which the reference uses).  Returns X (N, T, D) float64 and
    Y (N, n_labels, T) float64 -- the reference's ``samples[s][0]`` and ``samples[s][3]``."""
    assert num_labeled_states <= num_possible_states
    assert n_lags == 2, "the reference generator supports exactly 2 lags (data_utils.py:94)"
    if num_possible_states > num_labeled_states:
        num_labeled_states += 1
    if noise_type not in ("gaussian", "white"):
        raise ValueError("noise_type %r (superpositional noise is deprecated in the reference)" % noise_type)
    rs = np.random if rng is None else rng
    A = np.asarray(lagged_adj_graphs, dtype=np.float64)
    S, T, N = num_possible_states, recording_length, num_samples
    mu = np.asarray(noise_mu, dtype=np.float64).reshape(D)
    var = np.asarray(noise_var, dtype=np.float64).reshape(D)
    amp = np.asarray(innovation_amp_coeffs, dtype=np.float64).reshape(D)
    cos2 = np.array([2 * np.cos(2 * np.pi * np.asarray(base_freqs, dtype=np.float64).reshape(D)[i]) for i in range(D)])
    a = np.mean(innovation_amp_coeffs)
    n_steps = T + burnin_period            # recursion steps after X_t0, X_t1
    # ---- random numbers, in the reference's stream order --------------------------------
    x0 = np.empty((N, S, D))
    g = np.empty((N, S, n_steps + 1, D))
    w0 = np.empty((N, S))
    w1 = np.empty((N, S))
    noise = np.empty((N, D * T))
    for s in range(N):
        for k in range(S):
            x0[s, k] = rs.uniform(-1 * a, a, D)
            g[s, k] = rs.standard_normal((n_steps + 1) * D).reshape(n_steps + 1, D)
            w0[s, k] = rs.uniform()
            w1[s, k] = rs.uniform()
        if noise_type == "white":
            noise[s] = rs.uniform(-1 * a, a, D * T)
        else:
            noise[s] = rs.normal(np.mean(noise_mu), np.mean(noise_var) * a, D * T)
    innov = mu + var * g                    # np.random.normal(mu[i], var[i]) = mu + var * gauss
    # ---- the recursion, every (recording, state) chain at once ---------------------------
    C = N * S
    Ac = np.broadcast_to(A[None], (N,) + A.shape).reshape(C, D, D, A.shape[-1])
    codes = None
    if activation_codes is not None:
        ac = np.asarray(activation_codes)
        codes = np.broadcast_to(ac[None], (N,) + ac.shape).reshape(C, D, D, ac.shape[-1])
    innov = innov.reshape(C, n_steps + 1, D)
    h0 = x0.reshape(C, D)
    h1 = _chain_step(h0, h0, Ac, codes, cos2, amp, innov[:, 0], num_lags=1)
    keep = np.empty((C, T, D))
    hm2, hm1 = h0, h1
    for n in range(n_steps):
        hn = _chain_step(hm1, hm2, Ac, codes, cos2, amp, innov[:, n + 1], num_lags=n_lags)
        if n >= burnin_period:
            keep[:, n - burnin_period] = hn
        hm2, hm1 = hm1, hn
    sig = keep.reshape(N, S, T, D).transpose(0, 1, 3, 2)      # (N, S, D, T)
    # ---- state weighting, labels, additive noise -----------------------------------------
    X = np.zeros((N, D, T))
    true_lab = np.zeros((N, num_labeled_states, T))
    for k in range(S):
        w = np.stack([np.linspace(w0[s, k], w1[s, k], T) for s in range(N)])   # (N, T)
        X = X + sig[:, k] * w[:, None, :]
        row = k if k < num_labeled_states - 1 else num_labeled_states - 1
        true_lab[:, row] = true_lab[:, row] + w
    true_lab[:, -1] = true_lab[:, -1] / (1. * (S - (num_labeled_states - 1)))
    if label_type == "Oracle":
        Y = np.zeros((N, num_labeled_states, T)) + true_lab
    elif label_type == "OneHot":
        Y = np.zeros((N, num_labeled_states, T))
        idx = np.argmax(true_lab, axis=1)                          # (N, T)
        np.put_along_axis(Y, idx[:, None, :], 1., axis=1)
    else:
        raise ValueError("Unrecognized LABEL_TYPE==" + str(label_type))
    X = X + noise_amp_coeffs * noise.reshape(N, D, T)
    return X.transpose(0, 2, 1).copy(), Y


class NormalizedWindowSet:
    """NormalizedSyntheticWVARDataset over in-memory recordings.

    recordings: sequence of (T, D) float64 arrays (the reference's ``sample[0]``, file
    order); labels: matching (K, T) arrays.  Attributes mirror the reference:
    ``channel_means`` (1, D) float64 numpy, ``channel_std_devs`` (1, D) float64 torch,
    ``data`` = the kept recording indices after the shuffle / grid-search cut.
    ``grid_fraction`` is the grid-search cut (4: the synthetic quarter, 10: the LFP tenth,
    None: no cut, DREAM4); ``fortran_sums`` reproduces the synthetic recordings' memory layout
    in the statistics (the reference stores ``curr_samp.T``), False sums the arrays as given."""

    def __init__(self, recordings, labels, shuffle=True, shuffle_seed=0, grid_search=True, grid_fraction=4,
                 fortran_sums=True):
        self.recordings = [np.asarray(r) for r in recordings]
        self.labels = [np.asarray(y) for y in labels]
        accepted = [i for i, r in enumerate(self.recordings) if not np.isnan(np.sum(r))]
        if not accepted:
            raise ValueError("no finite recordings")
        T, D = self.recordings[accepted[0]].shape
        self.num_time_steps, self.num_chans = T, D
        lay = np.asfortranarray if fortran_sums else (lambda a: a)
        summed = None
        for i in accepted:                       # synthetic_datasets.py:66-73 (sequential sum)
            summed = self.recordings[i] if summed is None else summed + self.recordings[i]
        n = len(accepted)
        # the reference's synthetic recordings are ``curr_samp.T`` (Fortran-ordered, kept
        # by pickle) and numpy's reduction order follows the memory layout: sum the same way
        self.channel_means = (np.sum(lay(summed), axis=0) / (1. * n * T)).reshape(1, D)
        sq = None
        for i in accepted:                       # :89-104
            d2 = (self.recordings[i] - self.channel_means) ** 2.
            sq = d2 if sq is None else sq + d2
        self.channel_std_devs = torch.from_numpy(np.sqrt(np.sum(lay(sq), axis=0) / (1. * n * T))).reshape(1, D)
        self.data = list(accepted)
        if shuffle:
            random.Random(shuffle_seed).shuffle(self.data)
        if grid_search and grid_fraction:
            self.data = self.data[:len(self.data) // grid_fraction]

    def __len__(self):
        return len(self.data)

    def __getitem__(self, index):
        """(x, y) as float32: x = (float32(recording) - mean) / std evaluated in float64
        (torch promotion against the float64 statistics), as the reference does."""
        i = self.data[index]
        x = torch.from_numpy(self.recordings[i]).squeeze().to(torch.float32)
        x = (x - torch.from_numpy(self.channel_means)) / self.channel_std_devs
        return x.to(torch.float32), torch.from_numpy(self.labels[i]).to(torch.float32)

    def materialize(self, device=None, dtype=torch.float32):
        """All kept windows, normalised, as (N, T, D) and (N, K, T) tensors on ``device``
        (one host->device copy; the fit loop then slices batches in HBM)."""
        xs = torch.from_numpy(np.stack([self.recordings[i] for i in self.data])).to(torch.float32)
        xs = (xs - torch.from_numpy(self.channel_means)) / self.channel_std_devs
        ys = torch.from_numpy(np.stack([self.labels[i] for i in self.data]))
        return xs.to(device=device, dtype=dtype), ys.to(device=device, dtype=dtype)

    def batches(self, batch_size, device=None, dtype=torch.float32):
        """The DataLoader(batch_size) sequence (in order, last partial batch kept) as
        device-resident views."""
        X, Y = self.materialize(device, dtype)
        return [(X[i:i + batch_size], Y[i:i + batch_size]) for i in range(0, X.shape[0], batch_size)]


# --------------------------------------------------------------------------- subset-pickle directories
_FILE_FILTERS = {
    "dream4": lambda x: "subset_" in x,                      # dream4_datasets.py:38
    "lfp": lambda x: "_subset" in x,                         # local_field_potential_datasets.py:40
    "synthetic": lambda x: "_subset" in x or "subset_" in x,  # synthetic_datasets.py:41
}
_GRID_FRACTION = {"dream4": None, "lfp": 10, "synthetic": 4}


def average_regions(signal, average_region_map):
    """local_field_potential_datasets.py:118-132: (T, C) -> (T, R) float64, region r the mean of
    its listed channels, regions in the map's key order."""
    out = np.zeros((signal.shape[0], len(average_region_map)))
    for i, name in enumerate(average_region_map.keys()):
        out[:, i] = np.mean(signal[:, average_region_map[name]], axis=1)
    return out


def _load_subset_file(path):
    """One subset file of the reference's curated data sets: a pickled list of
    (x (T, C), y, ...) samples written by the user's data-curation scripts."""
    with open(path, "rb") as fh:
        return pickle.load(fh)


class NormalizedRecordingDirectory(NormalizedWindowSet):
    """The reference's per-directory normalised data sets (DREAM4, LFP, synthetic subsets).

    ``file_order`` overrides ``os.listdir(data_path)`` (the reference's file order, which is the
    filesystem's); the remaining arguments follow the reference constructors.  Only the
    ``"original"`` signal format is on the fitting path (directed-spectrum / flattened formats
    feed other model families)."""

    def __init__(self, data_path, kind="dream4", shuffle=True, shuffle_seed=0, grid_search=True,
                 average_region_map=None, signal_format="original", file_order=None):
        if kind not in _FILE_FILTERS:
            raise ValueError("kind must be one of %s" % sorted(_FILE_FILTERS))
        if signal_format != "original":
            raise NotImplementedError("signal_format %r is not on the REDCLIFF-S fitting path" % signal_format)
        if average_region_map is not None and kind != "lfp":
            raise ValueError("average_region_map applies to LFP data sets only")
        names = list(os.listdir(data_path)) if file_order is None else list(file_order)
        self.files = [x for x in names if _FILE_FILTERS[kind](x) and ".pkl" in x and "metadata" not in x]
        self.data_path, self.kind, self.average_region_map = data_path, kind, average_region_map
        recs, labs, self.sources = [], [], []
        x_ind, y_ind = 0, (3 if kind == "synthetic" else 1)
        for name in self.files:
            for j, smp in enumerate(_load_subset_file(os.path.join(data_path, name))):
                x = np.asarray(smp[x_ind])
                if kind == "synthetic" and x.ndim > 2:
                    x = x[0]
                if average_region_map is not None:
                    x = average_regions(x, average_region_map)
                recs.append(x)
                labs.append(np.asarray(smp[y_ind]))
                self.sources.append((os.path.join(data_path, name), j))
        super().__init__(recs, labs, shuffle=shuffle, shuffle_seed=shuffle_seed, grid_search=grid_search,
                         grid_fraction=_GRID_FRACTION[kind], fortran_sums=False)

    def source(self, index):
        """(file path, position in file) of item ``index`` -- the reference's ``data[index]``."""
        return self.sources[self.data[index]]


def _split_dirs(data_root_path, train_portion, name_filter):
    """The loaders' one-time train / validation split of a root directory's subset files
    (dream4_datasets.py:168-183, local_field_potential_datasets.py:198-213): the first
    train_portion of os.listdir's subset files are copied to ``train``, the rest to ``validation``."""
    train_path, val_path = os.path.join(data_root_path, "train"), os.path.join(data_root_path, "validation")
    if not os.path.exists(train_path):
        assert not os.path.exists(val_path)
        os.mkdir(train_path)
        os.mkdir(val_path)
        files = [x for x in os.listdir(data_root_path) if name_filter(x) and ".pkl" in x]
        cut = int(train_portion * len(files))
        for f in files[:cut]:
            shutil.copy(os.path.join(data_root_path, f), os.path.join(train_path, f))
        for f in files[cut:]:
            shutil.copy(os.path.join(data_root_path, f), os.path.join(val_path, f))
    return train_path, val_path


def load_normalized_DREAM4_data_train_test_split(data_root_path, batch_size, shuffle=True, shuffle_seed=0,
                                                 train_portion=0.8, grid_search=True, device=None):
    """dream4_datasets.py:168-189 -> (train batches, validation batches), device-resident."""
    tp, vp = _split_dirs(data_root_path, train_portion, lambda x: "subset_" in x)
    return tuple(NormalizedRecordingDirectory(p, "dream4", shuffle, shuffle_seed, grid_search).batches(batch_size, device)
                 for p in (tp, vp))


def load_normalized_lfp_data_train_test_split(data_root_path, batch_size, shuffle=True, shuffle_seed=0,
                                              train_portion=0.8, grid_search=True, average_region_map=None,
                                              device=None):
    """local_field_potential_datasets.py:198-219 -> (train batches, validation batches).  The
    reference copies files whose names contain ``subset_`` here but its data set then reads only
    ``*_subset*`` names (:40 vs :207); both filters are kept as written."""
    tp, vp = _split_dirs(data_root_path, train_portion, lambda x: "subset_" in x)
    return tuple(NormalizedRecordingDirectory(p, "lfp", shuffle, shuffle_seed, grid_search, average_region_map)
                 .batches(batch_size, device) for p in (tp, vp))
