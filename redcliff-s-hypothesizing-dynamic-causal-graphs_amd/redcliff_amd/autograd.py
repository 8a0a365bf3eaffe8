"""Autograd at the drop-in boundary.

The reference's modules return graph tensors: ``cMLP.forward`` (models/cmlp.py:90-101),
``cMLP.GC`` (:147-203), ``DGCNN_Embedder.forward`` (models/redcliff_factor_score_embedders.py:
366-388), ``REDCLIFF_S_CMLP*.forward`` (...withStateSmoothing.py:388-412) and ``compute_loss``
(:624-731), whose result the reference itself calls ``.backward()`` on (:783).  External
training code does the same, so these stay differentiable here.

Each is a ``torch.autograd.Function``:
  * forward = the fused gfx950 kernels (the same launches the no-grad path uses; BatchNorm
    running statistics advance exactly as in the reference, once per embedder evaluation);
  * backward = a recomputation through the generic HIP-GEMM path (redcliff_amd.generic: every
    contraction in ``redcliff_gemm``, element-wise glue as torch ops on the GPU) followed by
    ``torch.autograd.grad``.  BatchNorm in the recomputation uses the same batch statistics
    (train mode) or running statistics (eval mode) without advancing them again.
The fused ``batch_update`` never builds a graph (it has its own fused backward); these are
for callers that train or differentiate through the public methods.
"""
import torch

from . import generic as G
from . import kernels


def grad_needed(tensors):
    return torch.is_grad_enabled() and any(isinstance(t, torch.Tensor) and t.requires_grad for t in tensors)


def _grads(outs, gouts, inputs):
    pairs = [(o, g) for o, g in zip(outs, gouts) if g is not None and o.requires_grad]
    if not pairs:
        return [None] * len(inputs)
    o, g = zip(*pairs)
    want = [t for t in inputs if t is not None and t.requires_grad]
    got = iter(torch.autograd.grad(o, want, g, allow_unused=True)) if want else iter(())
    return [next(got) if (t is not None and t.requires_grad) else None for t in inputs]


def _leaf(t, need):
    return t.detach().requires_grad_(bool(need))


# ----------------------------------------------------------------------------- cMLP / MLP
def _factor_params(cmlps):
    out = []
    for f in cmlps:
        for net in f.networks:
            out += [net.layers[0].weight, net.layers[0].bias, net.layers[1].weight, net.layers[1].bias]
    return out


def _windows(X, L):
    B, T, p = X.shape
    return X.unfold(1, L, 1).permute(0, 1, 3, 2).reshape(B * (T - L + 1), L, p)


class _CMLPForward(torch.autograd.Function):
    """cMLP.forward on sliding windows (models/cmlp.py:90-101): fused factor kernel forward,
    HIP-GEMM recomputation backward."""

    @staticmethod
    def forward(ctx, X, cmlps, *params):
        ctx.cmlps = cmlps
        # the parameters are saved too: an in-place change before backward (an optimizer step
        # between two backwards of a retained graph) trips autograd's version check, as stock
        # modules do, instead of silently differentiating the new values
        ctx.save_for_backward(X, *params)
        return torch.stack(kernels.cmlp_forward(list(cmlps), X.detach()), 0)  # (F, B, S, p)

    @staticmethod
    def backward(ctx, gout):
        X, *params = ctx.saved_tensors
        cmlps = ctx.cmlps
        with torch.enable_grad():
            Xr = _leaf(X, ctx.needs_input_grad[0])
            lp = [_leaf(p, p.requires_grad) for p in params]
            L = cmlps[0].networks[0].layers[0].weight.shape[2]
            B, T, p = Xr.shape
            win = _windows(Xr, L)
            outs = []
            i = 0
            for f in cmlps:
                nets = []
                for _ in f.networks:
                    nets.append(lp[i:i + 4])
                    i += 4
                y = _mlp_group_params(nets, win)  # (B*S, p)
                outs.append(y.view(B, T - L + 1, p))
            out = torch.stack(outs, 0)
            g = _grads([out], [gout], [Xr] + lp)
        return (g[0], None) + tuple(g[1:])


def _mlp_group_params(nets, Xw):
    """generic.mlp_group with explicit (W0, b0, W1, b1) tensors per network."""
    B, L, p = Xw.shape
    W0 = torch.stack([n[0] for n in nets])
    Gn, h = W0.shape[0], W0.shape[1]
    x = Xw.transpose(1, 2).reshape(1, B, p * L)
    z = G.bmm(x, W0.reshape(Gn, h, p * L).transpose(1, 2)) + torch.stack([n[1] for n in nets])[:, None, :]
    W1 = torch.stack([n[2] for n in nets])
    z = G.bmm(torch.relu(z), W1[..., 0].transpose(1, 2)) + torch.stack([n[3] for n in nets])[:, None, :]
    return z[..., 0].transpose(0, 1)


def cmlp_forward(cmlps, X):
    """[(B, T-L+1, p)] per cMLP, differentiable when gradients are requested."""
    params = _factor_params(cmlps)
    X = X.to(torch.float32)
    if grad_needed([X] + params):
        out = _CMLPForward.apply(X, tuple(cmlps), *params)
        return [out[i] for i in range(len(cmlps))]
    return kernels.cmlp_forward(list(cmlps), X)


# ----------------------------------------------------------------------------- group norms
class _GroupNorms(torch.autograd.Function):
    """G (F, p, p, L) = ||W0[:, c, t]||, G0 (F, p, p) = ||W0[:, c, :]|| (models/cmlp.py:147-167)
    of the layer-0 weights of F groups of p networks: kernel forward, analytic backward
    dW = W / G * dG (G > 0), as torch.norm's gradient."""

    @staticmethod
    def forward(ctx, cmlps, *W0s):
        Gs, G0s = kernels.cmlp_gc_norms(list(cmlps))
        ctx.save_for_backward(Gs, G0s, *W0s)
        return Gs, G0s

    @staticmethod
    def backward(ctx, gG, gG0):
        Gs, G0s = ctx.saved_tensors[:2]
        W0s = ctx.saved_tensors[2:]
        Fn, p = Gs.shape[0], Gs.shape[1]
        W = torch.stack(W0s).view(Fn, p, *W0s[0].shape)  # (F, p_out, h, p_in, L)
        out = torch.zeros_like(W)
        if gG is not None:
            Gb = Gs.unsqueeze(2)  # (F, p_out, 1, p_in, L)
            out = out + torch.where(Gb > 0, W / torch.where(Gb > 0, Gb, torch.ones_like(Gb)), torch.zeros_like(W)) \
                * gG.unsqueeze(2)
        if gG0 is not None:
            G0b = G0s.unsqueeze(2).unsqueeze(-1)  # (F, p_out, 1, p_in, 1)
            out = out + torch.where(G0b > 0, W / torch.where(G0b > 0, G0b, torch.ones_like(G0b)),
                                    torch.zeros_like(W)) * gG0.unsqueeze(2).unsqueeze(-1)
        grads = out.view(Fn * p, *W0s[0].shape)
        return (None,) + tuple(grads[i] for i in range(grads.shape[0]))


def group_norms(cmlps):
    """(G, G0) of a list of cMLPs, differentiable when gradients are requested."""
    W0s = [net.layers[0].weight for f in cmlps for net in f.networks]
    if grad_needed(W0s):
        return _GroupNorms.apply(tuple(cmlps), *W0s)
    return kernels.cmlp_gc_norms(list(cmlps))


# ----------------------------------------------------------------------------- REDCLIFF forward / embedder
def dgcnn_params(dg):
    return [dg.A] + [gc.weight for gc in dg.layer1.gc1] + [dg.BN1.weight, dg.BN1.bias, dg.fc1.linear.weight,
                                                           dg.fc1.linear.bias, dg.fc2.linear.weight, dg.fc2.linear.bias]


def _dgcnn_recompute(dg, params, x, train_bn, bn_stats=None):
    """torcheeg DGCNN forward on node features x (B, p, F) with explicit parameter tensors;
    BatchNorm with batch statistics (train) / running statistics (eval: `bn_stats`, the
    (running_mean, running_var) snapshot taken at forward time), never advancing them."""
    A, gcw = params[0], params[1:1 + dg.num_layers]
    bnw, bnb, f1w, f1b, f2w, f2b = params[1 + dg.num_layers:]
    bn = dg.BN1
    xt = x.transpose(1, 2)
    if train_bn:
        xt = torch.nn.functional.batch_norm(xt, None, None, bnw, bnb, True, 0.0, bn.eps)
    else:
        rm, rv = bn_stats if bn_stats is not None else (bn.running_mean, bn.running_var)
        xt = torch.nn.functional.batch_norm(xt, rm, rv, bnw, bnb, False, 0.0, bn.eps)
    xb = xt.transpose(1, 2)
    B = xb.shape[0]
    Ar = torch.relu(A)
    d = 1.0 / torch.sqrt(Ar.sum(1) + 1e-10)
    Lap = (d[:, None] * Ar) * d[None, :]
    sup = [None, Lap]
    for _ in range(2, dg.num_layers):
        sup.append(G.mm(sup[-1], Lap))
    res = None
    for i in range(dg.num_layers):
        ax = xb if i == 0 else G.bmm(sup[i].unsqueeze(0), xb)
        term = G.bmm(ax, gcw[i].unsqueeze(0))
        res = term if res is None else res + term
    r = torch.relu(res).reshape(1, B, -1)
    f1 = G.bmm(r, f1w.t().unsqueeze(0))[0] + f1b
    return G.bmm(torch.relu(f1).unsqueeze(0), f2w.t().unsqueeze(0))[0] + f2b


class _FusedForward(torch.autograd.Function):
    """REDCLIFF forward in the published mode (...withStateSmoothing.py:326-385): embedder once,
    K x p factor networks, x_sim = sum_k w_k y_k.  Outputs (x_sim (B, p), y (B, K, p),
    w_raw (B, K)); forward on the fused kernels (BatchNorm advanced once in train mode)."""

    @staticmethod
    def forward(ctx, X, model, train_bn, *params):
        eng = model.engine()
        bn = _bn_snapshot(model, train_bn)  # eval mode: the running statistics this forward used
        w_raw, y, xs = eng.forward_outputs(X.detach(), train_bn=train_bn, bn_updates=1)
        ctx.model, ctx.train_bn = model, train_bn
        ctx.save_for_backward(X, *params, *bn)
        return xs, y.contiguous(), w_raw

    @staticmethod
    def backward(ctx, gxs, gy, gw):
        X, *rest = ctx.saved_tensors
        m = ctx.model
        params, bn = (rest, None) if ctx.train_bn else (rest[:-2], tuple(rest[-2:]))
        with torch.enable_grad():
            Xr = _leaf(X, ctx.needs_input_grad[0])
            lp = [_leaf(p, p.requires_grad) for p in params]
            xs, y, w = _fused_recompute(m, Xr, lp, ctx.train_bn, bn)
            g = _grads([xs, y, w], [gxs, gy, gw], [Xr] + lp)
        return (g[0], None, None) + tuple(g[1:])


def fused_params(model):
    dg = model.factor_score_embedder.dgcnn.dgcnn
    return dgcnn_params(dg) + _factor_params(model.factors)


def _bn_snapshot(model, train_bn):
    """() in train mode (batch statistics); else copies of the BatchNorm running statistics as
    the forward sees them, so a later train-mode forward advancing them cannot change an earlier
    eval-mode graph's backward."""
    if train_bn:
        return ()
    bn = model.factor_score_embedder.dgcnn.dgcnn.BN1
    return (bn.running_mean.detach().clone(), bn.running_var.detach().clone())


def _fused_recompute(m, X, lp, train_bn, bn_stats=None):
    dg = m.factor_score_embedder.dgcnn.dgcnn
    ne = 1 + dg.num_layers + 6
    F, L, K, p = m.embed_lag, m.gen_lag, m.num_factors_nK, m.num_series
    w = _dgcnn_recompute(dg, lp[:ne], X[:, X.shape[1] - F:, :].transpose(1, 2), train_bn, bn_stats)
    fp = lp[ne:]
    nets = [fp[4 * i:4 * i + 4] for i in range(K * p)]
    y = _mlp_group_params(nets, X[:, X.shape[1] - L:, :]).view(X.shape[0], K, p)
    emb = m.factor_score_embedder
    weff = torch.sigmoid(emb.sigmoid_eccentricity_coeff * w) if emb.use_sigmoid_restriction else w
    xs = None
    for k in range(K):
        t = weff[:, k:k + 1] * y[:, k, :]
        xs = t if xs is None else xs + t
    return xs, y, w


def fused_forward(model, Xw, train_bn):
    """(x_sim (B, p), y (B, K, p), w_raw (B, K)) of windows Xw (B, Lmax, p); a graph when needed."""
    params = fused_params(model)
    if grad_needed([Xw] + params):
        return _FusedForward.apply(Xw, model, train_bn, *params)
    w_raw, y, xs = model.engine().forward_outputs(Xw, train_bn=train_bn, bn_updates=1)
    return xs, y, w_raw


class _EmbedderForward(torch.autograd.Function):
    """DGCNN_Embedder.forward through the owning model's fused embedder launch; w_raw (B, K)."""

    @staticmethod
    def forward(ctx, Xw, model, train_bn, *params):
        eng = model.engine()
        bn = _bn_snapshot(model, train_bn)
        w_raw, _, _ = eng.forward_outputs(Xw.detach(), train_bn=train_bn, bn_updates=1)
        ctx.model, ctx.train_bn = model, train_bn
        ctx.save_for_backward(Xw, *params, *bn)
        return w_raw

    @staticmethod
    def backward(ctx, gw):
        Xw, *rest = ctx.saved_tensors
        m = ctx.model
        dg = m.factor_score_embedder.dgcnn.dgcnn
        params, bn = (rest, None) if ctx.train_bn else (rest[:-2], tuple(rest[-2:]))
        with torch.enable_grad():
            Xr = _leaf(Xw, ctx.needs_input_grad[0])
            lp = [_leaf(p, p.requires_grad) for p in params]
            F = m.embed_lag
            w = _dgcnn_recompute(dg, lp, Xr[:, Xr.shape[1] - F:, :].transpose(1, 2), ctx.train_bn, bn)
            g = _grads([w], [gw], [Xr] + lp)
        return (g[0], None, None) + tuple(g[1:])


def embedder_forward(model, Xw, train_bn):
    """Raw DGCNN embedder output w (B, K) of time-major windows Xw (B, Lmax, p)."""
    params = dgcnn_params(model.factor_score_embedder.dgcnn.dgcnn)
    if grad_needed([Xw] + params):
        return _EmbedderForward.apply(Xw, model, train_bn, *params)
    w_raw, _, _ = model.engine().forward_outputs(Xw, train_bn=train_bn, bn_updates=1)
    return w_raw


def standalone_dgcnn_forward(dg, x):
    """DGCNN_Embedder without an owning REDCLIFF model: the generic HIP-GEMM path (differentiable,
    BatchNorm module semantics)."""
    return G.dgcnn_forward(dg, x.to(torch.float32))
