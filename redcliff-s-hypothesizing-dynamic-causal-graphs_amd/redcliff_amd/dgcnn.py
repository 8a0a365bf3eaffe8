"""DGCNN modules with the parameter tree of torcheeg 1.1.3 ``DGCNN`` and of the reference's
``DGCNN_Model`` wrapper (models/dgcnn.py:15-61).

Only the parameter tree and the initialisation order live here (so that a seeded model
is identical to the reference's); the arithmetic runs in the gfx950 kernels of
csrc/rc_embed.hip, driven by redcliff_amd.engine.  Keys produced by ``state_dict()``:
``dgcnn.A``, ``dgcnn.layer1.gc1.{i}.weight``, ``dgcnn.BN1.*``, ``dgcnn.fc1.linear.*``,
``dgcnn.fc2.linear.*`` -- identical to the reference checkpoints.
"""
import torch
import torch.nn as nn

M1 = 64  # torcheeg DGCNN fc1 width


class GraphConvolution(nn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.weight = nn.Parameter(torch.empty(in_channels, out_channels))
        nn.init.xavier_normal_(self.weight)
        self.bias = None


class Chebynet(nn.Module):
    def __init__(self, in_channels, num_layers, out_channels):
        super().__init__()
        self.num_layers = num_layers
        self.gc1 = nn.ModuleList([GraphConvolution(in_channels, out_channels) for _ in range(num_layers)])


class Linear(nn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.linear = nn.Linear(in_channels, out_channels)
        nn.init.xavier_normal_(self.linear.weight)
        nn.init.zeros_(self.linear.bias)


class DGCNN(nn.Module):
    """torcheeg.models.DGCNN(in_channels, num_electrodes, num_layers, hid_channels, num_classes).

    Registration order (= RNG order): layer1 (Chebynet), BN1, fc1, fc2, A."""

    def __init__(self, in_channels=5, num_electrodes=62, num_layers=2, hid_channels=32, num_classes=2):
        super().__init__()
        self.in_channels = in_channels
        self.num_electrodes = num_electrodes
        self.num_layers = num_layers
        self.hid_channels = hid_channels
        self.num_classes = num_classes
        self.layer1 = Chebynet(in_channels, num_layers, hid_channels)
        self.BN1 = nn.BatchNorm1d(in_channels)
        self.fc1 = Linear(num_electrodes * hid_channels, M1)
        self.fc2 = Linear(M1, num_classes)
        self.A = nn.Parameter(torch.empty(num_electrodes, num_electrodes))
        nn.init.xavier_normal_(self.A)


class DGCNN_Model(nn.Module):
    """models/dgcnn.py:15-61 (the baseline fit/batch_update of that file are out of scope)."""

    def __init__(self, num_channels, num_wavelets_per_chan, num_features_per_node, num_graph_conv_layers,
                 num_hidden_nodes, num_classes):
        super().__init__()
        self.num_channels = num_channels
        self.num_wavelets_per_chan = num_wavelets_per_chan
        self.num_nodes = num_channels * num_wavelets_per_chan
        self.num_features_per_node = num_features_per_node
        self.num_graph_conv_layers = num_graph_conv_layers
        self.num_hidden_nodes = num_hidden_nodes
        self.num_classes = num_classes
        self.supervised_loss_fn = nn.MSELoss(reduction="mean")
        self.dgcnn = DGCNN(num_features_per_node, self.num_nodes, num_graph_conv_layers, num_hidden_nodes, num_classes)

    def GC(self, threshold=True, combine_node_feature_edges=False):
        """models/dgcnn.py:47-61: raw A^T; with combine=True the Frobenius norm of each
        1x1 (wavelet) block, i.e. |A|^T."""
        G = self.dgcnn.A
        if combine_node_feature_edges:
            w = self.num_wavelets_per_chan
            if w == 1:
                G = torch.abs(G)
            else:
                p = self.num_channels
                G = torch.linalg.vector_norm(G.reshape(p, w, p, w), dim=(1, 3))
        G = G.T
        return (G > 0).int() if threshold else G
