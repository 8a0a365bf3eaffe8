"""MI355X-native REDCLIFF-S cMLP factor-model fitting path.

Drop-in classes for the reference's models/ modules; compute in libredcliff_hip.so
(gfx950 HIP kernels, C-ABI in include/redcliff_hip.h)."""
from .cmlp import MLP, cMLP
from .dgcnn import DGCNN, DGCNN_Model
from .redcliff_factor_score_embedders import (DGCNN_Embedder, MLPClassifierForMultipleObjectives,
                                              MLPClassifierForSingleObjective, cEmbedder)
from .redcliff_s_cmlp import REDCLIFF_S_CMLP
from .redcliff_s_cmlp_withStateSmoothing import REDCLIFF_S_CMLP_withStateSmoothing
from .replicas import PerReplica, ReplicaPack, fit_packs, grid_packs, shard_grid
from .data_parallel import DataParallelFit

__all__ = ["MLP", "cMLP", "DGCNN", "DGCNN_Model", "DGCNN_Embedder", "cEmbedder", "MLPClassifierForSingleObjective",
           "MLPClassifierForMultipleObjectives", "REDCLIFF_S_CMLP", "REDCLIFF_S_CMLP_withStateSmoothing", "ReplicaPack",
           "PerReplica", "fit_packs", "grid_packs", "shard_grid", "DataParallelFit"]
