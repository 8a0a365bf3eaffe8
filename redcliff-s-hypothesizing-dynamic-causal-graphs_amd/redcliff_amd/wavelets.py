"""Wavelet-decomposed inputs (``wavelet_level != None``).

With ``wavelet_level = l`` every channel arrives as l + 1 wavelet series, so the model works on
``num_series = num_chans * (l + 1)`` series: the factor networks, the cEmbedder networks and
the DGCNN nodes are simply that many (the HIP kernels see p = num_series).  What is specific to
wavelets is GC post-processing, restated here from the reference:

* ranking masks built at construction (models/cmlp.py:61-78 for the factors,
  models/redcliff_factor_score_embedders.py:207-224 for the cEmbedder; both assert 4 wavelets
  per channel, i.e. l = 3), applied by ``GC(rank_wavelets=True)``;
* ``GC(combine_wavelet_representations=True)`` sums blocks of the estimate into a
  (num_chans, num_chans[, lag]) matrix (models/cmlp.py:179-200, embedders.py:307-326).  The
  reference indexes those blocks with a stride of ``wavelet_level`` (not l + 1) and this
  restatement keeps that.

The masks are built with the reference's exact tensor operations (same float32 roundings);
the post-processing runs on the device of the estimate.
"""
import torch


def _submask(rows, wavelets_per_chan):
    """The reference's per-channel block: rows x wavelets_per_chan factors 1.3^(2 (r - i))."""
    rank_factor = wavelets_per_chan // 4
    sub = torch.ones(rows, wavelets_per_chan)
    for i in range(rows):
        sub[i, :] = sub[i, :] * (1.3 ** (2. * (rank_factor - 1. * i)))
    for i in range(wavelets_per_chan):
        sub[:, i] = sub[:, i] * (1.3 ** (2. * (rank_factor - 1. * i)))
    return sub


def factor_mask(num_chans, wavelet_level):
    """(num_series, num_series) ranking mask of a cMLP (models/cmlp.py:61-78)."""
    num_series = int(num_chans * (wavelet_level + 1))
    mask = torch.ones(num_series, num_series)
    wpc = int(num_series / num_chans)
    assert wpc == 4  # the reference implements 4 wavelets per channel only
    sub = _submask(wpc, wpc)
    for i in range(num_series // wpc):
        for j in range(num_series // wpc):
            mask[wpc * i:wpc * (i + 1), wpc * j:wpc * (j + 1)] = sub * mask[wpc * i:wpc * (i + 1), wpc * j:wpc * (j + 1)]
    return mask


def embedder_mask(num_chans, num_factor_preds, wavelet_level):
    """(num_factor_preds, num_series) ranking mask of a cEmbedder
    (models/redcliff_factor_score_embedders.py:207-224)."""
    num_series = int(num_chans * (wavelet_level + 1))
    mask = torch.ones(num_factor_preds, num_series)
    wpc = int(num_series / num_chans)
    assert wpc == 4
    sub = _submask(1, wpc)
    for i in range(num_factor_preds):
        for j in range(num_series // wpc):
            mask[i:i + 1, wpc * j:wpc * (j + 1)] = sub * mask[i:i + 1, wpc * j:wpc * (j + 1)]
    return mask


def gc_post(GC, mask, wavelet_level, num_chans, num_series, lag, ignore_lag, combine, rank):
    """Rank and / or combine one GC estimate exactly as cMLP.GC / cEmbedder.GC do before
    thresholding (models/cmlp.py:169-200)."""
    if rank:
        assert mask is not None
        mask = mask.to(GC.device)
        if ignore_lag:
            GC = mask * GC
        else:
            assert GC.shape == (num_series, num_series, lag)
            GC = GC.clone()
            for l in range(lag):
                GC[:, :, l] = mask * GC[:, :, l]
    if wavelet_level is not None and combine:
        wl = wavelet_level
        if not ignore_lag:
            assert len(GC.size()) == 3
            out = torch.zeros((num_chans, num_chans, lag), device=GC.device)
            for r in range(num_chans):
                for c in range(num_chans):
                    sl = GC[r * wl:(r + 1) * wl, c * wl:(c + 1) * wl, :]
                    out[r, c, :] = out[r, c, :] + torch.sum(torch.sum(sl, 0, keepdim=True), 1, keepdim=True)[0, 0, :]
        else:
            out = torch.zeros((num_chans, num_chans), device=GC.device)
            for r in range(num_chans):
                for c in range(num_chans):
                    out[r, c] = out[r, c] + torch.sum(GC[r * wl:(r + 1) * wl, c * wl:(c + 1) * wl])
        GC = out
    return GC
