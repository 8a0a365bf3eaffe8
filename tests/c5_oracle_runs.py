"""Oracle trajectories of the C5 stress-config error-budget test (tests/test_gpu_parity.py), one per
worker process so the five CPU runs proceed side by side while the GPU runs the HIP path.
TEST INFRASTRUCTURE ONLY (imports oracle/)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

LR = 5e-4


class Float64Default:
    def __enter__(self):
        self.prev = torch.get_default_dtype()
        torch.set_default_dtype(torch.float64)

    def __exit__(self, *exc):
        torch.set_default_dtype(self.prev)


class FlipNearTies:
    """Run the float64 oracle with every near-tie DECISION of the path taken the other way.

    The path has data-dependent discrete decisions: the ReLU gates of the graph convolution,
    fc1 and the factor hidden layers, and the sign of every term of the fw-L1 and lag-weighted
    adjacency-L1 norms (the gradient of |v| is sign(v)).  Where a decision's argument is within
    fp32 rounding of zero (|v| <= tau * max|v| of its tensor), any fp32 implementation -- the
    reference's own CPU path included -- may take either branch, and the branch moves the Adam
    update of the affected weights by up to ~lr (eps-normalised steps).  This context patches
    torch.relu / F.relu / the L1 torch.norm so that every such decision is flipped; the
    difference between this run and the plain float64 run bounds what tie resolution alone can
    change.  ``self.flipped`` counts the flipped decisions.  Tie bands follow the fp32 error of
    each decision's argument: the factor hidden pre-activations are p*L = 1280-term contractions
    (on the matrix cores in the HIP path) and the L1 sign arguments v = w_bk G_k + A^T carry the
    error of the whole embedder forward in w (a 6400-term fc1 contraction), ~1e-6 relative; the
    embedder's ReLU arguments are held to 1e-7."""

    def __init__(self, tau_factor=1e-6, tau_embedder=1e-7, tau_l1=1e-6):
        self.tau = {"factor relu": tau_factor, "embedder relu": tau_embedder, "l1": tau_l1}
        self.flipped = dict((k, 0) for k in self.tau)

    def _near(self, z, kind):
        zz = z.detach().abs()
        m = (zz <= self.tau[kind] * zz.max()) & (zz > 0) if zz.numel() else zz > 0
        self.flipped[kind] += int(m.sum())
        return m

    def __enter__(self):
        import torch.nn.functional as F_
        self.saved = (torch.relu, F_.relu, torch.norm)
        norm0 = torch.norm

        def relu_factor(z):  # torch.relu: the factor networks' hidden layer (OMLP.forward)
            return z * ((z.detach() > 0) ^ self._near(z, "factor relu")).to(z.dtype)

        def relu_embedder(z, inplace=False):  # F.relu: graph convolution, fc1, normalize_A (torcheeg DGCNN)
            return z * ((z.detach() > 0) ^ self._near(z, "embedder relu")).to(z.dtype)

        def norm(x, p="fro", dim=None, keepdim=False, out=None, dtype=None):
            if p == 1 and dim is None and not keepdim:
                s = torch.sign(x.detach())
                s = torch.where(self._near(x, "l1"), -s, s)
                return (x * s).sum()
            return norm0(x, p, dim, keepdim, out, dtype)

        torch.relu, F_.relu, torch.norm = relu_factor, relu_embedder, norm
        return self

    def __exit__(self, *exc):
        import torch.nn.functional as F_
        torch.relu, F_.relu, torch.norm = self.saved


class PermutedContraction:
    """The oracle's factor layer-0 contraction (Conv1d over p channels x L lags, OMLP.forward)
    with its input channels taken in a permuted order: the same mathematics, another fp32
    summation order of the pre-activations z.  Window permutations (perm<s>) only reorder the
    batch reductions; this realisation varies what the HIP path varies too (the matrix-core
    k-order of the p*L-term contraction), so near-tie hidden-unit gates can fall either way."""

    def __init__(self, p, seed):
        self.perm = torch.from_numpy(np.random.RandomState(seed).permutation(p))

    def __enter__(self):
        from oracle import redcliff_oracle as R
        self.saved = R.OMLP.forward
        perm = self.perm

        def forward(mod, X):
            z = X.transpose(2, 1)
            for i, layer in enumerate(mod.layers):
                if i == 0:
                    z = torch.nn.functional.conv1d(z[:, perm, :], layer.weight[:, perm, :], layer.bias)
                else:
                    z = layer(torch.relu(z))
            return z.transpose(2, 1)
        R.OMLP.forward = forward
        return self

    def __exit__(self, *exc):
        from oracle import redcliff_oracle as R
        R.OMLP.forward = self.saved


class GateMargins:
    """Records, for every factor hidden unit (k, j, u), the smallest relative distance of its
    pre-activation from the ReLU threshold over every window of every training step:
    min |z_bu| / max |z| of its network.  A unit whose margin is within fp32 resolution of the
    trajectory is a near-tie gate: another fp32 implementation may take the other branch."""

    def __init__(self, model):
        self.ids = {}
        for k, f in enumerate(model.factors):
            for j, net in enumerate(f.networks):
                self.ids[id(net)] = (k, j)
        K, p = len(model.factors), len(model.factors[0].networks)
        h = model.factors[0].networks[0].layers[0].weight.shape[0]
        self.margin = np.full((K, p, h), np.inf)
        self.on = False

    def __enter__(self):
        from oracle import redcliff_oracle as R
        self.saved = R.OMLP.forward
        rec = self

        def forward(mod, X):
            z = mod.layers[0](X.transpose(2, 1))
            if rec.on and id(mod) in rec.ids:
                zz = z.detach().abs()
                m = (zz / zz.max().clamp_min(1e-300)).amin(dim=(0, 2)).double().numpy()
                k, j = rec.ids[id(mod)]
                rec.margin[k, j] = np.minimum(rec.margin[k, j], m)
            for layer in mod.layers[1:]:
                z = layer(torch.relu(z))
            return z.transpose(2, 1)
        R.OMLP.forward = forward
        return self

    def __exit__(self, *exc):
        from oracle import redcliff_oracle as R
        R.OMLP.forward = self.saved


def build_oracle(cfg, seed=0):
    from oracle.redcliff_oracle import OracleREDCLIFF, reference_coeffs
    coeff = reference_coeffs(cfg["K"], cfg["p"])
    eargs = [("num_features_per_node", cfg["F"]), ("num_graph_conv_layers", cfg["n"]),
             ("num_hidden_nodes", cfg["H"]), ("sigmoid_eccentricity_coeff", 10.0)]
    args = (cfg["p"], cfg["L"], [cfg["h"]], cfg["F"], [0], cfg["L"], 1, cfg["K"], cfg["nsup"], coeff, False, "DGCNN",
            eargs, "conditional_factor_fixed_embedder", "apply_factor_weights_after_sim_completion")
    kw = dict(num_sims=1, training_mode="pretrain_embedder_then_acclimate_factors_then_combined",
              num_pretrain_epochs=1, num_acclimation_epochs=1)
    torch.manual_seed(seed)
    return OracleREDCLIFF(*args, **kw)


def gc_of(mod, Xin):
    g = mod.GC("conditional_factor_fixed_embedder", X=Xin, threshold=False, ignore_lag=True)
    return np.stack([np.stack([e.detach().cpu().numpy() for e in row]) for row in g]).astype(np.float64)


def trajectory(kind, cfg, X, Y, Xv, Yv, nb, threads=3):
    """One oracle realisation of the schedule (pretrain, acclimate, combined; nb batches of
    cfg["B"] windows each): kind "fp32", "perm<s>" (rows of every batch permuted with seed s),
    "chperm<s>" (the factor contraction's channel order permuted, PermutedContraction), "fp64"
    or "fp64flip".  Returns its state (numpy), validation values, lag-free GC on the
    first 8 validation windows and the flipped-decision counts."""
    from oracle.redcliff_oracle import make_optimizers
    torch.set_num_threads(threads)
    X, Y, Xv, Yv = (torch.from_numpy(np.asarray(a)) for a in (X, Y, Xv, Yv))
    B = cfg["B"]
    o = build_oracle(cfg)
    dbl = kind.startswith("fp64")
    if dbl:
        o = o.double()
    perm = None
    if kind.startswith("perm"):
        perm = torch.from_numpy(np.random.RandomState(100 + int(kind[4:])).permutation(B))
    flip = FlipNearTies() if kind == "fp64flip" else None
    ctx = Float64Default() if dbl else _Null()
    cperm = PermutedContraction(cfg["p"], 200 + int(kind[6:])) if kind.startswith("chperm") else _Null()
    gates = GateMargins(o) if kind == "fp64" else None
    with ctx, cperm, (gates if gates is not None else _Null()):
        oA, oB = make_optimizers(o, LR, 1e-4, 1e-4, LR, 1e-4, 1e-4)
        if gates is not None:
            gates.on = True
        with (flip if flip is not None else _Null()):
            for epoch in (0, 1, 2):
                for bi in range(nb):
                    Xb, Yb = X[bi * B:(bi + 1) * B], Y[bi * B:(bi + 1) * B]
                    if perm is not None:
                        Xb, Yb = Xb[perm], Yb[perm]
                    if dbl:
                        Xb, Yb = Xb.double(), Yb.double()
                    o.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
        if gates is not None:
            gates.on = False
        val = o.validate([(Xv.double(), Yv.double()) if dbl else (Xv, Yv)])
        o.eval()
        Lm = max(cfg["L"], cfg["F"])
        Xg = Xv[:8, :Lm]
        with torch.no_grad():
            g = gc_of(o, Xg.double() if dbl else Xg)
    sd = dict((k, v.detach().numpy().copy()) for k, v in o.state_dict().items() if not k.startswith("gen_model."))
    return dict(state=sd, val=dict((k, float(v)) for k, v in val.items()), gc=g,
                flipped=None if flip is None else dict(flip.flipped),
                gate_margin=None if gates is None else gates.margin)


class _Null:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False
