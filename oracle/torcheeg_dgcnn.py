"""TEST INFRASTRUCTURE ONLY -- restatement of torcheeg 1.1.3 ``torcheeg.models.DGCNN``.

The reference builds its factor-score embedder on ``torcheeg.models.DGCNN``
(``/root/reference/models/dgcnn.py:9,37-43``; version pin ``redcliffs-env.yml:129``,
``torcheeg==1.1.3``).  torcheeg is NOT installed in this image and is NOT vendored in
the reference, so its arithmetic is restated here from the package's published
algorithm:

* ``BatchNorm1d(in_channels)`` applied to ``x.transpose(1, 2)``;
* ``normalize_A``: ReLU, row-sum degree ``d``, ``d^-1/2`` with a 1e-10 guard, ``D A D``;
* Chebyshev supports ``[I, L, L@L, ...]`` (``generate_cheby_adj``);
* ``GraphConvolution``: ``(adj @ x) @ W`` with no bias, ``xavier_normal_`` init;
* ``Linear``: ``nn.Linear`` followed by ``xavier_normal_`` weight / zero bias;
* ``fc1(num_electrodes * hid -> 64)``, ReLU, ``fc2(64 -> num_classes)``;
* ``A = xavier_normal_(num_electrodes, num_electrodes)``, registered LAST.

Parameter registration (and therefore RNG-consumption) order: layer1.gc1.{i}.weight,
BN1, fc1, fc2, A.  Everything that depends on this file is marked
"parity unpinned at the torcheeg 1.1.3 boundary": the reference repository has no test
or fixture that pins the DGCNN arithmetic.

This module is used (a) as the ``sys.modules['torcheeg.models']`` stub when the golden
fixtures are generated from the reference in this container and (b) by the CPU oracle.
It is never imported by the product package.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


class GraphConvolution(nn.Module):
    def __init__(self, in_channels, out_channels, bias=False):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.weight = nn.Parameter(torch.FloatTensor(in_channels, out_channels))
        nn.init.xavier_normal_(self.weight)
        self.bias = None
        if bias:
            self.bias = nn.Parameter(torch.FloatTensor(out_channels))
            nn.init.zeros_(self.bias)

    def forward(self, x, adj):
        out = torch.matmul(torch.matmul(adj, x), self.weight)
        return out if self.bias is None else out + self.bias


class Linear(nn.Module):
    def __init__(self, in_channels, out_channels, bias=True):
        super().__init__()
        self.linear = nn.Linear(in_channels, out_channels, bias=bias)
        nn.init.xavier_normal_(self.linear.weight)
        if bias:
            nn.init.zeros_(self.linear.bias)

    def forward(self, inputs):
        return self.linear(inputs)


def normalize_A(A, symmetry=False):
    A = F.relu(A)
    if symmetry:
        A = A + torch.transpose(A, 0, 1)
    d = torch.sum(A, 1)
    d = 1 / torch.sqrt(d + 1e-10)
    D = torch.diag_embed(d)
    return torch.matmul(torch.matmul(D, A), D)


def generate_cheby_adj(A, num_layers):
    support = []
    for i in range(num_layers):
        if i == 0:
            support.append(torch.eye(A.shape[1]).to(A.device))
        elif i == 1:
            support.append(A)
        else:
            support.append(torch.matmul(support[-1], A))
    return support


class Chebynet(nn.Module):
    def __init__(self, in_channels, num_layers, out_channels):
        super().__init__()
        self.num_layers = num_layers
        self.gc1 = nn.ModuleList([GraphConvolution(in_channels, out_channels) for _ in range(num_layers)])

    def forward(self, x, L):
        adj = generate_cheby_adj(L, self.num_layers)
        result = None
        for i, gc in enumerate(self.gc1):
            if i == 0:
                result = gc(x, adj[i])
            else:
                result += gc(x, adj[i])
        return F.relu(result)


class DGCNN(nn.Module):
    def __init__(self, in_channels=5, num_electrodes=62, num_layers=2, hid_channels=32, num_classes=2):
        super().__init__()
        self.in_channels = in_channels
        self.num_electrodes = num_electrodes
        self.hid_channels = hid_channels
        self.num_layers = num_layers
        self.num_classes = num_classes
        self.layer1 = Chebynet(in_channels, num_layers, hid_channels)
        self.BN1 = nn.BatchNorm1d(in_channels)
        self.fc1 = Linear(num_electrodes * hid_channels, 64)
        self.fc2 = Linear(64, num_classes)
        self.A = nn.Parameter(torch.FloatTensor(num_electrodes, num_electrodes))
        nn.init.xavier_normal_(self.A)

    def forward(self, x):
        x = self.BN1(x.transpose(1, 2)).transpose(1, 2)
        L = normalize_A(self.A)
        result = self.layer1(x, L)
        result = result.reshape(x.shape[0], -1)
        result = F.relu(self.fc1(result))
        return self.fc2(result)
