"""cMLP factor networks (models/cmlp.py) backed by the gfx950 kernels.

Parameter tree and initialisation order are the reference's (``networks.{j}.layers.{i}``;
Conv1d(p, h, L) default init, then ``xavier_uniform_``, then the 1x1 Conv1d,
models/cmlp.py:13-27) so seeded models are bit-identical.  ``forward``, ``GC`` and
``perform_prox_update_on_GC_weights`` run on the GPU through libredcliff_hip.so
(redcliff_factor_forward / redcliff_gc_norms / redcliff_prox); there is no CPU path.
"""
import torch
import torch.nn as nn

from . import kernels, wavelets


class MLP(nn.Module):
    def __init__(self, num_series, lag, hidden):
        super().__init__()
        self.activation = torch.nn.ReLU()
        self.lag = lag
        widths = list(hidden) + [1]
        first = nn.Conv1d(num_series, widths[0], lag)
        nn.init.xavier_uniform_(first.weight)
        self.layers = nn.ModuleList([first] + [nn.Conv1d(a, b, 1) for a, b in zip(widths[:-1], widths[1:])])

    def forward(self, X):
        """X (B, T, p) -> (B, T - lag + 1, 1) (models/cmlp.py:29-35).  Without gradients: the
        grouped factor kernel (one network == a one-output cMLP); with gradients: the generic
        HIP-GEMM path (a graph through redcliff_gemm)."""
        from . import autograd as AG
        params = [t for layer in self.layers for t in (layer.weight, layer.bias)]
        if AG.grad_needed([X] + params):
            from .generic import mlp_group
            kernels.require_gpu(X, "MLP.forward")
            L = self.layers[0].weight.shape[2]
            B, T, p = X.shape
            win = AG._windows(X.to(torch.float32), L)
            return mlp_group([self], win).view(B, T - L + 1, 1)
        return kernels.single_network_forward(self, X)


class cMLP(nn.Module):
    def __init__(self, num_chans, lag, hidden, wavelet_level=None, save_path=None):
        """wavelet_level = l: num_chans * (l + 1) wavelet series and the ranking mask of
        models/cmlp.py:57-82 (redcliff_amd.wavelets; the mask heat-map plot is not drawn)."""
        super().__init__()
        self.num_chans = num_chans
        self.wavelet_level = wavelet_level
        self.lag = lag
        self.hidden = list(hidden)
        if wavelet_level is None:
            self.num_series = num_chans
            self.wavelet_mask = None
        else:
            self.num_series = int(num_chans * (wavelet_level + 1))
            self.wavelet_mask = wavelets.factor_mask(num_chans, wavelet_level)
        self.activation = torch.nn.ReLU()
        self.networks = nn.ModuleList([MLP(self.num_series, lag, hidden) for _ in range(self.num_series)])

    def forward(self, X):
        """X (batch, T, p) -> (batch, T - lag + 1, p) (models/cmlp.py:90-101); a graph tensor when
        gradients are requested (fused kernel forward, HIP-GEMM backward: redcliff_amd.autograd)."""
        from . import autograd as AG
        return AG.cmlp_forward([self], X)[0]

    def perform_prox_update_on_GC_weights(self, lam, lr, penalty):
        """In-place GL / GSGL / H proximal step on layer-0 weights (models/cmlp.py:117-144)."""
        kernels.cmlp_prox([self], lam, lr, penalty)

    def GC(self, threshold=True, ignore_lag=True, combine_wavelet_representations=False, rank_wavelets=False):
        """Group norms of layer-0 weights: (p, p) or (p, p, lag), then the wavelet ranking /
        combination and the threshold (models/cmlp.py:147-203)."""
        from . import autograd as AG
        G, G0 = AG.group_norms([self]) if not threshold else kernels.cmlp_gc_norms([self])
        out = G0[0] if ignore_lag else G[0]
        out = self.gc_post(out, ignore_lag, combine_wavelet_representations, rank_wavelets)
        return (out > 0).int() if threshold else out

    def gc_post(self, G, ignore_lag, combine, rank):
        """Ranking mask and wavelet combination of one (un-thresholded) estimate."""
        if not rank and not (self.wavelet_level is not None and combine):
            return G
        return wavelets.gc_post(G, self.wavelet_mask, self.wavelet_level, self.num_chans, self.num_series, self.lag,
                                ignore_lag, combine, rank)
