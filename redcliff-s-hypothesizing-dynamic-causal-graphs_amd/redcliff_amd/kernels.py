"""Thin torch-tensor wrappers around the C-ABI for the stand-alone cMLP operations.

Every function here requires CUDA (ROCm) tensors and raises otherwise: the compute runs
in libredcliff_hip.so, never on the CPU.
"""
import ctypes

import torch

from . import _native as nat


def current_stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def require_gpu(t, what):
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise RuntimeError("%s runs on the MI355X only (HIP kernels); move the model/tensors to 'cuda'" % what)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def factor_dims(K, p, L, h, Bmax=1, R=1):
    return nat.Dims(R=R, Bmax=Bmax, T=L, p=p, L=L, K=K, h=h, F=L, n=1, H=1, M1=1, nsup=0, use_sigmoid=0,
                    sigmoid_ecc=0.0)


def factor_layout(K, p, h, L):
    kp = K * p
    o = {"W0": 0}
    o["b0"] = o["W0"] + kp * h * p * L
    o["W1"] = o["b0"] + kp * h
    o["b1"] = o["W1"] + kp * h
    o["total"] = o["b1"] + kp
    return o


def factor_views(flat, cmlps, p, h, L):
    """(param, view) pairs mapping each cMLP parameter onto the packed factor layout
    W0[K][p][h][p][L] | b0[K][p][h] | W1[K][p][h] | b1[K][p]."""
    K = len(cmlps)
    o = factor_layout(K, p, h, L)
    pairs = []
    for k, f in enumerate(cmlps):
        for j, net in enumerate(f.networks):
            kj = k * p + j
            l0, l1 = net.layers[0], net.layers[1]
            pairs.append((l0.weight, flat[o["W0"] + kj * h * p * L:o["W0"] + (kj + 1) * h * p * L].view(h, p, L)))
            pairs.append((l0.bias, flat[o["b0"] + kj * h:o["b0"] + (kj + 1) * h]))
            pairs.append((l1.weight, flat[o["W1"] + kj * h:o["W1"] + (kj + 1) * h].view(1, h, 1)))
            pairs.append((l1.bias, flat[o["b1"] + kj:o["b1"] + kj + 1]))
    return pairs


def _check_single_hidden(cmlps):
    for f in cmlps:
        for net in f.networks:
            if len(net.layers) != 2:
                raise NotImplementedError("the gfx950 factor kernels cover gen_hidden of length 1 (one hidden layer)")


def pack_factors(cmlps):
    """Gather the parameters of ``cmlps`` (same shapes) into a fresh packed device buffer."""
    _check_single_hidden(cmlps)
    f0 = cmlps[0]
    W = f0.networks[0].layers[0].weight
    require_gpu(W, "cMLP")
    h, p, L = W.shape
    flat = torch.empty(factor_layout(len(cmlps), p, h, L)["total"], device=W.device, dtype=torch.float32)
    with torch.no_grad():
        for prm, view in factor_views(flat, cmlps, p, h, L):
            view.copy_(prm.detach())
    return flat, (p, h, L)


def cmlp_gc_norms(cmlps):
    """G[k] (p, p, L) and G0[k] (p, p): norms of layer-0 weights (models/cmlp.py:162-166)."""
    flat, (p, h, L) = pack_factors(cmlps)
    K = len(cmlps)
    dims = factor_dims(K, p, L, h)
    G = torch.empty(K, p, p, L, device=flat.device, dtype=torch.float32)
    G0 = torch.empty(K, p, p, device=flat.device, dtype=torch.float32)
    nat.check(nat.lib().redcliff_gc_norms(ctypes.byref(dims), ptr(flat), flat.numel(), ptr(G), ptr(G0),
                                          current_stream()), "gc_norms")
    return G, G0


def cmlp_prox(cmlps, lam, lr, penalty):
    code = {"GL": 0, "GSGL": 1, "H": 2}.get(penalty)
    if code is None:
        raise ValueError("unsupported penalty: %s" % penalty)
    flat, (p, h, L) = pack_factors(cmlps)
    dims = factor_dims(len(cmlps), p, L, h)
    nat.check(nat.lib().redcliff_prox(ctypes.byref(dims), ptr(flat), flat.numel(), float(lam), float(lr), code,
                                      current_stream()), "prox")
    with torch.no_grad():
        for prm, view in factor_views(flat, cmlps, p, h, L):
            prm.copy_(view)


def factor_forward_packed(flat, K, p, h, L, Xwin):
    """y[b][k][j] for windows Xwin (B, L, p) (contiguous, on the GPU)."""
    B = Xwin.shape[0]
    out = torch.empty(B, K, p, device=Xwin.device, dtype=torch.float32)
    chunk = 512
    for b0 in range(0, B, chunk):
        nb = min(chunk, B - b0)
        dims = factor_dims(K, p, L, h, Bmax=nb)
        ws_floats = nat.lib().redcliff_factor_forward_workspace_floats(ctypes.byref(dims), nb)
        if ws_floats == 0:
            nat.check(-1, "factor_forward_workspace_floats")
        ws = torch.empty(ws_floats, device=Xwin.device, dtype=torch.float32)
        xw = Xwin[b0:b0 + nb].contiguous()
        nat.check(nat.lib().redcliff_factor_forward(ctypes.byref(dims), nb, ptr(xw), 0, ptr(flat), 0, ptr(ws),
                                                    ws_floats, ptr(out[b0:b0 + nb]), nb * K * p, current_stream()),
                  "factor_forward")
    return out


def cmlp_forward(cmlps, X):
    """Sliding-window forward of each cMLP: X (B, T, p) -> [(B, T-L+1, p)] (models/cmlp.py:90-101)."""
    require_gpu(X, "cMLP.forward")
    flat, (p, h, L) = pack_factors(cmlps)
    X = X.to(torch.float32)
    B, T, _ = X.shape
    S = T - L + 1
    if S < 1:
        raise ValueError("input shorter than the lag")
    win = X.unfold(1, L, 1).permute(0, 1, 3, 2).reshape(B * S, L, p).contiguous()
    y = factor_forward_packed(flat, len(cmlps), p, h, L, win).view(B, S, len(cmlps), p)
    return [y[:, :, k, :] for k in range(len(cmlps))]


def single_network_forward(mlp, X):
    """MLP.forward (models/cmlp.py:29-35): network output (B, T-L+1, 1)."""
    require_gpu(X, "MLP.forward")
    W = mlp.layers[0].weight
    h, p, L = W.shape
    if len(mlp.layers) != 2:
        raise NotImplementedError("the gfx950 factor kernels cover one hidden layer")
    # a one-network factor: pack as K=1, p_out=1 by replicating into a p-network layout
    flat = torch.zeros(factor_layout(1, p, h, L)["total"], device=W.device, dtype=torch.float32)
    o = factor_layout(1, p, h, L)
    with torch.no_grad():
        flat[o["W0"]:o["W0"] + h * p * L] = W.detach().reshape(-1)
        flat[o["b0"]:o["b0"] + h] = mlp.layers[0].bias.detach()
        flat[o["W1"]:o["W1"] + h] = mlp.layers[1].weight.detach().reshape(-1)
        flat[o["b1"]:o["b1"] + 1] = mlp.layers[1].bias.detach()
    X = X.to(torch.float32)
    B, T, _ = X.shape
    S = T - L + 1
    win = X.unfold(1, L, 1).permute(0, 1, 3, 2).reshape(B * S, L, p).contiguous()
    y = factor_forward_packed(flat, 1, p, h, L, win).view(B, S, p)
    return y[:, :, :1]
