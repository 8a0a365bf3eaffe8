"""Factor-score embedders (models/redcliff_factor_score_embedders.py).

``DGCNN_Embedder`` (the embedder of every published REDCLIFF-S run) is computed by the
fused gfx950 kernels through the owning REDCLIFF model's FitEngine.  ``cEmbedder`` and
the two "Vanilla" MLP classifiers keep the reference's parameter trees and seeded
initialisation so checkpoints and seeds stay interchangeable; they run (forward, GC and
training) on the generic HIP-GEMM path (redcliff_amd.generic).
"""
import torch
import torch.nn as nn

from . import wavelets
from .cmlp import MLP
from .dgcnn import DGCNN_Model


class DGCNN_Embedder(nn.Module):
    """models/redcliff_factor_score_embedders.py:335-392"""

    def __init__(self, num_channels, num_wavelets_per_chan, num_features_per_node, num_graph_conv_layers,
                 num_hidden_nodes, sigmoid_eccentricity_coeff, use_sigmoid_restriction, num_factors, num_classes):
        super().__init__()
        self.dgcnn = DGCNN_Model(num_channels, num_wavelets_per_chan, num_features_per_node, num_graph_conv_layers,
                                 num_hidden_nodes, num_factors)
        self.num_channels = num_channels
        self.num_wavelets_per_chan = num_wavelets_per_chan
        self.num_features_per_node = num_features_per_node
        self.num_graph_conv_layers = num_graph_conv_layers
        self.num_hidden_nodes = num_hidden_nodes
        self.num_factors = num_factors
        self.num_classes = num_classes
        self.use_sigmoid_restriction = use_sigmoid_restriction
        self.sigmoid = nn.Sigmoid() if use_sigmoid_restriction else None
        self.sigmoid_eccentricity_coeff = sigmoid_eccentricity_coeff if use_sigmoid_restriction else None
        self.owner = None  # set by the REDCLIFF model: the engine that evaluates this embedder

    def forward(self, X, use_final_activation=True):
        """(B, p, F) or (B, F, p) windows -> (factor weightings (B, K), class logits (B, nsup) | None).
        Inside a REDCLIFF model (the owner, re-attached after torch.load / deepcopy) the fused
        embedder launch evaluates it; a stand-alone embedder runs the generic HIP-GEMM path.
        Differentiable either way (redcliff_amd.autograd)."""
        assert X.dim() == 3
        if X.size(2) != self.num_features_per_node:  # (B, F, p) -> (B, p, F), as the reference (:369-371)
            assert X.size(1) == self.num_features_per_node
            X = torch.transpose(X, 1, 2)
        owner = self.owner() if self.owner is not None else None
        if owner is None:
            from .autograd import standalone_dgcnn_forward
            w = standalone_dgcnn_forward(self.dgcnn.dgcnn, X)
            logits = None
            if self.num_classes > 0:
                logits = w[:, :self.num_classes]
                if use_final_activation and self.use_sigmoid_restriction:
                    logits = torch.sigmoid(logits)
            if self.use_sigmoid_restriction:
                w = torch.sigmoid(self.sigmoid_eccentricity_coeff * w)
            return w, logits
        # X is (B, p, F) (nodes x features); the kernels read time-major windows (B, F, p)
        return owner._embed_windows(X.transpose(1, 2), use_final_activation)

    def GC(self, threshold=True, combine_node_feature_edges=False):
        return self.dgcnn.GC(threshold=threshold, combine_node_feature_edges=combine_node_feature_edges)

    def __getstate__(self):
        st = self.__dict__.copy()
        st["owner"] = None
        return st


class cEmbedder(nn.Module):
    """models/redcliff_factor_score_embedders.py:183-331."""

    def __init__(self, num_chans, num_class_preds, num_factor_preds, use_sigmoid_restriction,
                 sigmoid_eccentricity_coeff, lag, hidden, wavelet_level=None, save_path=None):
        super().__init__()
        self.num_chans = num_chans
        self.num_class_preds = num_class_preds
        self.num_factor_preds = num_factor_preds
        self.use_sigmoid_restriction = use_sigmoid_restriction
        self.sigmoid_eccentricity_coeff = sigmoid_eccentricity_coeff if use_sigmoid_restriction else None
        self.lag = lag
        self.hidden = hidden
        self.wavelet_level = wavelet_level
        if wavelet_level is None:
            self.num_series = num_chans
            self.wavelet_mask = None
        else:  # :206-224 (the mask heat-map plot is not drawn)
            self.num_series = int(num_chans * (wavelet_level + 1))
            self.wavelet_mask = wavelets.embedder_mask(num_chans, num_factor_preds, wavelet_level)
        self.save_path = save_path
        self.activation = torch.nn.ReLU()
        self.sigmoid = nn.Sigmoid() if use_sigmoid_restriction else None
        self.networks = nn.ModuleList([MLP(self.num_series, lag, hidden) for _ in range(num_factor_preds)])

    def forward(self, X, use_final_activation=True):
        """(B, lag, p) windows -> (w (B, K), class logits (B, nsup) | None) on the HIP GEMM."""
        from .generic import cembedder_forward
        return cembedder_forward(self, X, use_final_activation)

    def GC(self, threshold=True, ignore_lag=True, combine_wavelet_representations=False, rank_wavelets=False):
        from . import kernels
        W = torch.stack([net.layers[0].weight for net in self.networks])
        kernels.require_gpu(W, "cEmbedder.GC")
        # cEmbedder GC is the group norm of K networks over p inputs: one "factor" of K networks
        dims_owner = _Wrap(self.networks)
        G, G0 = kernels.cmlp_gc_norms([dims_owner])
        out = G0[0] if ignore_lag else G[0]
        out = self.gc_post(out, ignore_lag, combine_wavelet_representations, rank_wavelets)
        return (out > 0).int() if threshold else out

    def gc_post(self, G, ignore_lag, combine, rank):
        """Ranking mask and wavelet combination (models/redcliff_factor_score_embedders.py:297-326)."""
        if not rank and not (self.wavelet_level is not None and combine):
            return G
        return wavelets.gc_post(G, self.wavelet_mask, self.wavelet_level, self.num_chans, self.num_series, self.lag,
                                ignore_lag, combine, rank)


class _Wrap:
    """Adapter exposing K embedder MLPs as one cMLP-like group for the norm kernel."""

    def __init__(self, networks):
        self.networks = networks


class MLPClassifierForSingleObjective(nn.Module):
    """models/redcliff_factor_score_embedders.py:51-100 (forward on the HIP GEMM: redcliff_amd.generic)."""

    def __init__(self, num_series, num_in_timesteps, num_factor_scores, hidden_sizes, use_sigmoid_restriction,
                 sigmoid_eccentricity_coeff=10.):
        super().__init__()
        assert len(hidden_sizes) == 1
        self.num_series, self.num_in_timesteps, self.num_factor_scores = num_series, num_in_timesteps, num_factor_scores
        self.hidden_sizes = hidden_sizes
        self.flatten = nn.Flatten()
        self.use_sigmoid_restriction = use_sigmoid_restriction
        self.sigmoid = nn.Sigmoid() if use_sigmoid_restriction else None
        self.sigmoid_eccentricity_coeff = sigmoid_eccentricity_coeff if use_sigmoid_restriction else None
        kw = num_in_timesteps - ((num_in_timesteps - 1) % 2)
        self.series_embedding_layers = nn.Sequential(
            nn.Conv2d(1, hidden_sizes[0], (num_series, kw), stride=1, padding=(0, kw // 2), dilation=1, bias=False),
            nn.ReLU(),
            nn.Conv2d(hidden_sizes[0], hidden_sizes[0], (1, num_in_timesteps), stride=1, padding=0, dilation=1,
                      bias=False),
            nn.ReLU())
        self.unsup_factor_weighting_layer = nn.Linear(hidden_sizes[0], num_factor_scores, bias=False)
        self.num_out_classes = 0

    def forward(self, X, use_final_activation=True):
        from .generic import vanilla_forward
        return vanilla_forward(self, X, use_final_activation)


class MLPClassifierForMultipleObjectives(nn.Module):
    """models/redcliff_factor_score_embedders.py:104-179 (forward on the HIP GEMM: redcliff_amd.generic)."""

    def __init__(self, num_series, num_in_timesteps, num_factor_scores, num_out_classes, hidden_sizes,
                 use_sigmoid_restriction, sigmoid_eccentricity_coeff=10.):
        super().__init__()
        assert len(hidden_sizes) == 1
        self.num_series, self.num_in_timesteps = num_series, num_in_timesteps
        self.num_factor_scores, self.num_out_classes = num_factor_scores, num_out_classes
        self.hidden_sizes = hidden_sizes
        self.flatten = nn.Flatten()
        self.use_sigmoid_restriction = use_sigmoid_restriction
        self.sigmoid = nn.Sigmoid() if use_sigmoid_restriction else None
        self.sigmoid_eccentricity_coeff = sigmoid_eccentricity_coeff if use_sigmoid_restriction else None
        kw = num_in_timesteps - ((num_in_timesteps - 1) % 2)
        self.series_embedding_layers = nn.Sequential(
            nn.Conv2d(1, hidden_sizes[0], (num_series, kw), stride=1, padding=(0, kw // 2), dilation=1, bias=False),
            nn.ReLU(),
            nn.Conv2d(hidden_sizes[0], hidden_sizes[0], (1, num_in_timesteps), stride=1, padding=0, dilation=1,
                      bias=False),
            nn.ReLU())
        if num_factor_scores - num_out_classes > 0:
            self.unsup_factor_weighting_layer = nn.Linear(hidden_sizes[0] - num_out_classes,
                                                          num_factor_scores - num_out_classes, bias=False)
        else:
            self.unsup_factor_weighting_layer = None

    def forward(self, X, use_final_activation=True):
        from .generic import vanilla_forward
        return vanilla_forward(self, X, use_final_activation)
