"""Generic (non-fused) REDCLIFF-S path on the GPU.

The fused kernel chain (engine.py) covers the configuration every published run uses:
DGCNN embedder, num_sims == 1, factor weights applied after the simulation, one hidden
factor layer, embed_lag >= gen_lag, conditional_factor_fixed_embedder.  Everything else
the reference's classes accept runs here:

* cEmbedder and the Vanilla embedders (models/redcliff_factor_score_embedders.py:51-331);
* num_sims > 1 roll-outs on the factors' own predictions (...withStateSmoothing.py:326-385)
  and the smoothing penalty they make non-zero (:668-691);
* the per-step factor weighting forward mode (:253-323), which re-runs the embedder on
  simulated windows (gradients flow through BatchNorm's batch statistics);
* every GC estimation mode (:415-620), and several hidden factor layers.

Every contraction -- the K x p (or K) channel MLPs as one batched product, the DGCNN
Chebyshev powers, graph convolutions and fc layers, the Vanilla convolutions as im2col
products, the cEmbedder conditional GC products -- runs in ``redcliff_gemm`` (HIP, gfx950),
wrapped in an autograd Function whose backward is two more ``redcliff_gemm`` calls.  The
optimizer steps are ``redcliff_adam_apply`` (HipAdam: each group's parameters and Adam moments
are views of flat buffers, one gradient gather and one HIP launch per step).  The element-wise
glue (bias, ReLU, BatchNorm normalisation, losses) is torch operations on the GPU tensors.
There is no CPU path: tensors must be on the GPU and the HIP library must load.
"""
import ctypes
import math

import numpy as np
import torch
import torch.nn.functional as Fn

from . import _native as nat


# ----------------------------------------------------------------------------- HIP GEMM
def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _gemm(ta, tb, M, N, K, a, sa, b, sb, out, batch, lda, ldb):
    nat.check(nat.lib().redcliff_gemm(ta, tb, M, N, K, 1.0, a.data_ptr(), lda, sa, b.data_ptr(), ldb, sb, 0.0,
                                      out.data_ptr(), N, M * N, batch, _stream()), "gemm")


def _raw_bmm(a, b, ta=0, tb=0):
    """op(a[i]) @ op(b[i]) for 3-D contiguous fp32 CUDA tensors; a batch of 1 broadcasts."""
    Ba, Bb = a.shape[0], b.shape[0]
    Bc = max(Ba, Bb)
    M, K = (a.shape[2], a.shape[1]) if ta else (a.shape[1], a.shape[2])
    K2, N = (b.shape[2], b.shape[1]) if tb else (b.shape[1], b.shape[2])
    assert K == K2 and Ba in (1, Bc) and Bb in (1, Bc)
    out = torch.empty(Bc, M, N, device=a.device, dtype=torch.float32)
    _gemm(ta, tb, M, N, K, a, 0 if Ba == 1 else a.shape[1] * a.shape[2], b,
          0 if Bb == 1 else b.shape[1] * b.shape[2], out, Bc, a.shape[2], b.shape[2])
    return out


class _HipBmm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        a = a.contiguous()
        b = b.contiguous()
        ctx.save_for_backward(a, b)
        return _raw_bmm(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous()
        da = db = None
        if ctx.needs_input_grad[0]:
            da = _raw_bmm(g, b, tb=1)
            if a.shape[0] == 1 and da.shape[0] > 1:
                da = da.sum(0, keepdim=True)
        if ctx.needs_input_grad[1]:
            db = _raw_bmm(a, g, ta=1)
            if b.shape[0] == 1 and db.shape[0] > 1:
                db = db.sum(0, keepdim=True)
        return da, db


def bmm(a, b):
    """a (Ba, M, K) @ b (Bb, K, N) on the HIP GEMM (Ba, Bb in {1, max}); differentiable."""
    for t in (a, b):
        if not (t.is_cuda and t.dtype == torch.float32):
            raise RuntimeError("the generic REDCLIFF-S path runs on the MI355X in fp32 (HIP GEMM); got %s %s"
                               % (t.device, t.dtype))
    return _HipBmm.apply(a, b)


def mm(a, b):
    """2-D a (M, K) @ b (K, N)."""
    return bmm(a.unsqueeze(0), b.unsqueeze(0))[0]


# ----------------------------------------------------------------------------- building blocks
def mlp_group(nets, Xw):
    """G networks of models/cmlp.py:12-35 (lag-L Conv1d -> ReLU -> 1x1 Conv1d ...) on windows
    Xw (B, L, p) whose length equals the kernel width: returns (B, G)."""
    B, L, p = Xw.shape
    W0 = torch.stack([net.layers[0].weight for net in nets])  # (G, h, p, L)
    G, h = W0.shape[0], W0.shape[1]
    x = Xw.transpose(1, 2).reshape(1, B, p * L)  # q = c * L + t, the Conv1d weight order
    z = bmm(x, W0.reshape(G, h, p * L).transpose(1, 2)) + torch.stack([net.layers[0].bias for net in nets])[:, None, :]
    for i in range(1, len(nets[0].layers)):
        Wi = torch.stack([net.layers[i].weight for net in nets])  # (G, out, in, 1)
        bi = torch.stack([net.layers[i].bias for net in nets])
        z = bmm(torch.relu(z), Wi[..., 0].transpose(1, 2)) + bi[:, None, :]
    return z[..., 0].transpose(0, 1)  # (B, G)


def group_norms(weights, ignore_lag):
    """||W[:, c, t]|| over hidden units (and lags): models/cmlp.py:162-166, differentiable."""
    W = torch.stack(weights)  # (G, h, p, L)
    return torch.sqrt((W * W).sum(dim=(1, 3) if ignore_lag else 1))


def dgcnn_forward(g, x):
    """torcheeg 1.1.3 DGCNN (models/dgcnn.py:15-64) on node features x (B, p, F)."""
    B = x.shape[0]
    x = g.BN1(x.transpose(1, 2)).transpose(1, 2)
    A = torch.relu(g.A)
    d = 1.0 / torch.sqrt(A.sum(1) + 1e-10)
    Lap = (d[:, None] * A) * d[None, :]  # matmul(matmul(D, A), D) element by element
    n = g.num_layers
    supports = [None, Lap]
    for _ in range(2, n):
        supports.append(mm(supports[-1], Lap))
    result = None
    for i, gc in enumerate(g.layer1.gc1):
        ax = x if i == 0 else bmm(supports[i].unsqueeze(0), x)  # matmul(eye, x) == x
        term = bmm(ax, gc.weight.unsqueeze(0))
        result = term if result is None else result + term
    r = torch.relu(result).reshape(1, B, -1)
    f1 = bmm(r, g.fc1.linear.weight.t().unsqueeze(0))[0] + g.fc1.linear.bias
    return bmm(torch.relu(f1).unsqueeze(0), g.fc2.linear.weight.t().unsqueeze(0))[0] + g.fc2.linear.bias


def vanilla_embed(emb, X):
    """Conv2d(1,H,(p,kw)) -> ReLU -> Conv2d(H,H,(1,T)) -> ReLU of the Vanilla embedders
    (models/redcliff_factor_score_embedders.py:51-179) as im2col products: (B, H)."""
    B, T, p = X.shape
    c1, c2 = emb.series_embedding_layers[0], emb.series_embedding_layers[2]
    H, kw = c1.weight.shape[0], c1.weight.shape[3]
    cols = Fn.unfold(X.transpose(1, 2).reshape(B, 1, p, T), (p, kw), padding=(0, kw // 2))  # (B, p*kw, T')
    y1 = torch.relu(bmm(c1.weight.reshape(1, H, p * kw), cols))  # (B, H, T')
    y2 = bmm(y1.reshape(1, B, -1), c2.weight.reshape(H, -1).t().unsqueeze(0))[0]
    return torch.relu(y2)


def lin(layer, x):
    y = bmm(x.unsqueeze(0), layer.weight.t().unsqueeze(0))[0]
    return y if layer.bias is None else y + layer.bias


def cembedder_forward(emb, X, use_final_activation=True):
    """cEmbedder.forward (models/redcliff_factor_score_embedders.py:236-273): K channel MLPs over
    the window -> (factor weightings (B, K), class logits (B, nsup) | None)."""
    B = X.shape[0]
    w = mlp_group(list(emb.networks), X[:, -emb.lag:, :].contiguous()).reshape(B, emb.num_factor_preds)
    logits = None
    if emb.num_class_preds > 0:
        logits = w[:, :emb.num_class_preds]
        if use_final_activation and emb.use_sigmoid_restriction:
            logits = torch.sigmoid(logits)
    if emb.use_sigmoid_restriction:
        w = torch.sigmoid(emb.sigmoid_eccentricity_coeff * w)
    return w, logits


def vanilla_forward(emb, X, use_final_activation=True):
    """MLPClassifierForSingleObjective / ForMultipleObjectives.forward
    (models/redcliff_factor_score_embedders.py:51-179)."""
    B = X.shape[0]
    e = vanilla_embed(emb, X)
    sig, ecc = emb.use_sigmoid_restriction, emb.sigmoid_eccentricity_coeff
    n_cls = getattr(emb, "num_out_classes", 0)
    K = emb.num_factor_scores
    if n_cls > 0:
        sup = e[:, :n_cls]
        if emb.unsup_factor_weighting_layer is not None:
            w = torch.cat((sup, lin(emb.unsup_factor_weighting_layer, e[:, n_cls:]).view(B, K - n_cls)), 1)
        else:
            w = sup
        w = w.view(B, K)
        if sig:
            w = torch.sigmoid(ecc * w)
        logits = e[:, :n_cls]
        if use_final_activation and sig:
            logits = torch.sigmoid(logits)
        return w, logits
    w = lin(emb.unsup_factor_weighting_layer, e).view(B, K)
    return (torch.sigmoid(ecc * w) if sig else w), None


# ----------------------------------------------------------------------------- optimizer
class HipAdam:
    """One torch.optim.Adam (a single parameter group, coupled L2 weight decay -- the optimizers
    call_model_fit_method builds, general_utils/model_utils.py:747-762) stepped by
    ``redcliff_adam_apply`` (the same per-element update, in torch's operation order, as the
    fused chain's epilogues): the group's parameters become views of one flat buffer and the
    optimizer's ``exp_avg`` / ``exp_avg_sq`` / ``step`` state views of flat moment buffers and a
    shared step tensor, so ``optimizer.state_dict()`` round-trips and a step is one multi-tensor
    gradient gather plus one launch.  A step where some parameter has no gradient (torch skips
    those, weight decay included) or an option the kernel does not implement is left to
    ``optimizer.step()``."""

    def __init__(self, opt):
        self.opt = opt
        grp = opt.param_groups[0]
        self.params = list(grp["params"])
        self.released_for = None
        self.ok = (len(opt.param_groups) == 1 and not grp.get("amsgrad") and not grp.get("maximize")
                   and not grp.get("decoupled_weight_decay", False) and len(self.params) > 0
                   and all(p.is_cuda and p.dtype == torch.float32 for p in self.params))
        if not self.ok:
            return
        # one step count for the whole group: torch advances each parameter's own and skips those
        # without a gradient, so a torch-stepped optimizer whose parameters disagree stays with torch
        steps = set(int(float(st["step"])) if "step" in st else 0
                    for st in (opt.state.get(p) or {} for p in self.params))
        if len(steps) > 1:
            self.ok = False
            self.released_for = "unequal step counts %s" % sorted(steps)
            return
        dev = self.params[0].device
        n = sum(p.numel() for p in self.params)
        self.flat = torch.empty(n, device=dev, dtype=torch.float32)
        self.m = torch.zeros(n, device=dev, dtype=torch.float32)
        self.v = torch.zeros(n, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(n, device=dev, dtype=torch.float32)
        self.views, self.gviews = [], []
        o, t = 0, 0
        with torch.no_grad():
            for p in self.params:
                k = p.numel()
                view = self.flat[o:o + k].view_as(p)
                view.copy_(p.detach())
                st = opt.state.get(p)
                if st and "exp_avg" in st:  # a torch-stepped optimizer: continue from its moments
                    self.m[o:o + k].copy_(st["exp_avg"].reshape(-1))
                    self.v[o:o + k].copy_(st["exp_avg_sq"].reshape(-1))
                    t = int(float(st["step"]))
                p.data = view
                self.views.append((o, k))
                self.gviews.append(self.grad[o:o + k].view_as(p))
                o += k
        self.t = t
        self.step_t = torch.tensor(float(t), dtype=torch.float32)
        for p, (o, k) in zip(self.params, self.views):
            opt.state[p] = {"step": self.step_t, "exp_avg": self.m[o:o + k].view_as(p),
                            "exp_avg_sq": self.v[o:o + k].view_as(p)}
        self._hkey = None
        self._dims = nat.Dims(R=1, Bmax=1, T=1, p=1, L=1, K=1, h=1, F=1, n=1, H=1, M1=1, nsup=0, use_sigmoid=0,
                              sigmoid_ecc=0.0)

    def bound(self):
        return self.ok and all(p.data_ptr() == self.flat.data_ptr() + 4 * o for p, (o, _) in zip(self.params, self.views))

    def state_is_ours(self):
        """The optimizer's state still is this object's flat moments and shared step tensor
        (optimizer.load_state_dict() swaps in new tensors: then the loaded state must be taken)."""
        for p, (o, _) in zip(self.params, self.views):
            st = self.opt.state.get(p)
            if (not st or st.get("step") is not self.step_t
                    or st["exp_avg"].data_ptr() != self.m.data_ptr() + 4 * o
                    or st["exp_avg_sq"].data_ptr() != self.v.data_ptr() + 4 * o):
                return False
        return True

    def _hyper(self):
        g = self.opt.param_groups[0]
        key = (float(g["lr"]), tuple(float(b) for b in g["betas"]), float(g["eps"]), float(g["weight_decay"]))
        if key != self._hkey:
            h = nat.ReplicaHyper()
            h.A = nat.adam_hyper(*key)
            self._hdev = torch.from_numpy(np.frombuffer(bytes(h), dtype=np.uint8).copy()).to(self.flat.device)
            self._hkey = key
        return self._hdev

    def release(self):
        """Hand the optimizer back to torch: every parameter gets its own step tensor (torch's
        Adam advances each parameter's separately and skips those without a gradient); the moments
        stay views of the flat buffers."""
        if self.ok:
            for p in self.params:
                self.opt.state[p]["step"] = self.step_t.clone()
        self.ok = False

    def step(self):
        if not self.bound() or any(p.grad is None for p in self.params):
            self.released_for = "re-pointed parameters" if not self.bound() else "missing gradient"
            self.release()
            return self.opt.step()
        if int(float(self.step_t)) != self.t:  # stepped by torch in between (or its state edited)
            self.t = int(float(self.step_t))
        torch._foreach_copy_(self.gviews, [p.grad for p in self.params])
        n = self.flat.numel()
        nat.check(nat.lib().redcliff_adam_apply(ctypes.byref(self._dims), self.flat.data_ptr(), self.m.data_ptr(),
                                                self.v.data_ptr(), self.grad.data_ptr(), n, n,
                                                self._hyper().data_ptr(), 0, self.t + 1, _stream()), "adam_apply")
        self.t += 1
        self.step_t.fill_(float(self.t))


# ----------------------------------------------------------------------------- the model
class GenericPath:
    """forward / GC / compute_loss / batch_update / validate of one REDCLIFF-S model on the
    GPU through the HIP GEMM (see the module docstring)."""

    def __init__(self, model):
        self.m = model
        self._adams = {}

    def _step(self, opt):
        """opt.step() through HipAdam (one per optimizer object, built on its first step)."""
        h = self._adams.get(id(opt))
        reloaded = h is not None and h.opt is opt and h.ok and h.bound() and not h.state_is_ours()
        if h is None or h.opt is not opt or (h.ok and not h.bound()) or reloaded:
            if h is not None and h.opt is opt and not reloaded:
                h.release()  # its parameters were re-pointed: rebuild on the current ones
            # (after optimizer.load_state_dict() the rebuilt object continues from the loaded moments
            # and step count, which HipAdam.__init__ copies into its flat buffers)
            h = self._adams[id(opt)] = HipAdam(opt) if isinstance(opt, torch.optim.Adam) else None
        if h is None or not h.ok:  # released optimizers stay with torch (per-parameter step counts)
            return opt.step()
        return h.step()

    # -------------------------------------------------------------- embedder
    def embed(self, X, use_final_activation=True):
        """Embedder on the last embed_lag steps of X (B, T, p) (...withStateSmoothing.py:335-343)."""
        m = self.m
        emb = m.factor_score_embedder
        win = X[:, -m.embed_lag:, :]
        nsup = m.num_supervised_factors
        kind = m.factor_score_embedder_type
        if kind == "DGCNN":
            w = dgcnn_forward(emb.dgcnn.dgcnn, win.transpose(1, 2))
            logits = None
            if nsup > 0:
                logits = w[:, :nsup]
                if use_final_activation and emb.use_sigmoid_restriction:
                    logits = torch.sigmoid(logits)
            if emb.use_sigmoid_restriction:
                w = torch.sigmoid(emb.sigmoid_eccentricity_coeff * w)
            return w, logits
        return emb(win, use_final_activation)

    # -------------------------------------------------------------- factors
    def factor_step(self, cur):
        """All K x p channel networks on the last gen_lag steps of cur: list of K (B, 1, p)."""
        m = self.m
        nets = [net for f in m.factors for net in f.networks]
        y = mlp_group(nets, cur[:, -m.gen_lag:, :].contiguous())  # (B, K*p)
        B, p = cur.shape[0], m.num_series
        return [y[:, k * p:(k + 1) * p].unsqueeze(1) for k in range(m.num_factors_nK)]

    def forward(self, X, fw_given=None):
        m = self.m
        if m.forward_pass_mode == "apply_factor_weights_after_sim_completion":
            fw, logits = self.embed(X)
            if fw_given is not None:
                fw = fw_given
            if logits is None:
                logits = fw
            labels = [logits for _ in range(m.num_sims)]
            K = m.num_factors_nK
            outs = [[] for _ in range(K)]
            for s in range(m.num_sims):  # each factor rolls out on its own predictions (:350-374)
                step = self._rollout_step(outs, X, s)
                for k in range(K):
                    outs[k].append(step[k])
            per_factor = [torch.cat(o, dim=1) for o in outs]
            x_sim = None
            for k in range(K):
                term = fw[:, k].view(-1, 1, 1) * per_factor[k]
                x_sim = term if x_sim is None else x_sim + term
            return x_sim, per_factor, [fw], labels
        # apply_factor_weights_at_each_sim_step (:253-323)
        inputs = [X + 0.0]
        sims, preds_over, fws, labels = [], [], [], []
        for s in range(m.num_sims):
            if s > 0:
                last = sims[-1]
                inputs.append(last if last.size() == inputs[-1].size()
                              else torch.cat([inputs[-1][:, last.size(1):, :], last], dim=1))
            fw, logits = self.embed(inputs[s])
            if fw_given is not None:
                fw = fw_given
            labels.append(fw if logits is None else logits)
            fpreds = self.factor_step(inputs[s])
            combined = None
            for k in range(m.num_factors_nK):
                term = fw[:, k].view(-1, 1, 1) * fpreds[k]
                combined = term if combined is None else combined + term
            preds_over.append(fpreds)
            fws.append(fw)
            sims.append(combined)
        return torch.cat(sims, dim=1), preds_over, fws, labels

    def _rollout_step(self, outs, X, s):
        """Step s of every factor's roll-out: factor k's window is the original window with its own
        s previous predictions appended (cat(cur[:, 1:], prev), :355-371)."""
        m = self.m
        K, p = m.num_factors_nK, m.num_series
        if s == 0:
            return self.factor_step(X[:, -m.gen_lag:, :])
        ys = []
        nets_all = [list(f.networks) for f in m.factors]
        for k in range(K):
            cur = X[:, -m.gen_lag:, :] + 0.0
            for prev in outs[k][:s]:
                cur = prev if prev.size() == cur.size() else torch.cat([cur[:, prev.size(1):, :], prev], dim=1)
            y = mlp_group(nets_all[k], cur[:, -m.gen_lag:, :].contiguous())  # (B, p)
            ys.append(y.unsqueeze(1))
        return ys

    # -------------------------------------------------------------- GC
    def factor_gcs(self, threshold, ignore_lag, combine=False, rank=False):
        """cMLP.GC of every factor: norms, wavelet ranking / combination (models/cmlp.py:169-200),
        threshold, (n, n, 1) when lag-free (:450-454)."""
        out = []
        for f in self.m.factors:
            G = f.gc_post(group_norms([net.layers[0].weight for net in f.networks], ignore_lag), ignore_lag, combine,
                          rank)
            if G.dim() != 3:
                G = G.view(G.size(0), G.size(0), 1)
            out.append((G > 0).int() if threshold else G)
        return out

    def raw_embedder_gc(self, threshold, ignore_lag, combine, rank=False):
        m = self.m
        emb = m.factor_score_embedder
        if m.factor_score_embedder_type == "cEmbedder":
            G = emb.gc_post(group_norms([net.layers[0].weight for net in emb.networks], ignore_lag), ignore_lag, combine,
                            rank)
            if G.dim() != 3:
                assert G.size(0) == m.num_factors_nK  # :476 (a combined wavelet graph fails here, as in the reference)
                G = G.view(m.num_factors_nK, G.size(1), 1)
        elif m.factor_score_embedder_type == "DGCNN":
            G = emb.dgcnn.GC(threshold=False, combine_node_feature_edges=combine)  # models/dgcnn.py:47-61
            assert G.size(0) == m.num_series  # :472
            G = G.reshape(m.num_series, m.num_series, 1)
        else:
            raise ValueError("raw_embedder GC needs a causal embedder (cEmbedder / DGCNN)")
        return (G > 0).int() if threshold else G

    def fixed_embedder_gc(self, threshold, ignore_lag, combine, rank=False):
        G = self.raw_embedder_gc(threshold, ignore_lag, combine, rank)
        if self.m.factor_score_embedder_type == "DGCNN":
            return G
        assert G.size(0) == self.m.num_factors_nK  # :513
        Gt = G.float().transpose(0, 2).contiguous()  # (L, p, K): sum_k g_k g_k^T per lag (:514)
        out = bmm(Gt, Gt.transpose(1, 2)).transpose(0, 2)
        return out.int() if threshold else out

    def GC(self, mode, X=None, threshold=True, ignore_lag=True, combine=False, rank=False):
        m = self.m
        ls = min(m.gen_lag, m.embed_lag)
        K = m.num_factors_nK
        if mode == "fixed_factor_exclusive":
            return [self.factor_gcs(threshold, ignore_lag, combine, rank)]
        if mode == "raw_embedder":
            return [[self.raw_embedder_gc(threshold, ignore_lag, combine, rank)]]
        if mode == "fixed_embedder_exclusive":
            return [[self.fixed_embedder_gc(threshold, ignore_lag, combine, rank)]]
        if mode == "conditional_factor_exclusive":
            fw, _ = self.embed(X)
            fg = self.factor_gcs(threshold, ignore_lag, combine, rank)
            return [[fw[b, k] * fg[k] for k in range(fw.size(1))] for b in range(fw.size(0))]
        if mode == "conditional_embedder_exclusive":
            if m.factor_score_embedder_type == "DGCNN":
                raise ValueError("conditional_embedder_exclusive is not supported for model with DGCNN factor "
                                 "score embedder type")
            raw = self.raw_embedder_gc(threshold, ignore_lag, combine, rank).float()
            assert raw.size(0) == K  # :532
            nv, nl = raw.size(1), raw.size(2)
            fw, _ = self.embed(X)
            prods = []
            for k in range(K):
                g = raw[k].view(1, nv, nl).transpose(0, 2).contiguous()
                prods.append(bmm(g, g.transpose(1, 2)).transpose(0, 2))
            return [[fw[b, k] * prods[k] for k in range(fw.size(1))] for b in range(fw.size(0))]
        if mode == "fixed_factor_fixed_embedder":
            fg = self.factor_gcs(threshold, ignore_lag, combine, rank)
            eg = self.fixed_embedder_gc(threshold, ignore_lag, combine, rank)
            if not ignore_lag:
                return [[g[:, :, -ls:] + eg[:, :, -ls:] for g in fg]]
            return [[g + eg for g in fg]]
        if mode == "conditional_factor_fixed_embedder":
            cond = self.GC("conditional_factor_exclusive", X, threshold, ignore_lag, combine, rank)
            eg = self.fixed_embedder_gc(threshold, ignore_lag, combine, rank)
            return [[(c + eg) if ignore_lag else (c[:, :, -ls:] + eg[:, :, -ls:]) for c in row] for row in cond]
        if mode == "fixed_factor_conditional_embedder":
            fg = self.factor_gcs(threshold, ignore_lag, combine, rank)
            cond = self.GC("conditional_embedder_exclusive", X, threshold, ignore_lag, combine, rank)
            return [[(c + fg[k]) if ignore_lag else (c[:, :, -ls:] + fg[k][:, :, -ls:]) for k, c in enumerate(row)]
                    for row in cond]
        if mode == "conditional_factor_conditional_embedder":
            a = self.GC("conditional_factor_exclusive", X, threshold, ignore_lag, combine, rank)
            e = self.GC("conditional_embedder_exclusive", X, threshold, ignore_lag, combine, rank)
            return [[(a[b][k] + e[b][k]) if ignore_lag else (a[b][k][:, :, -ls:] + e[b][k][:, :, -ls:])
                     for k in range(K)] for b in range(len(a))]
        raise ValueError("GC EST MODE == " + str(mode) + " IS NOT SUPPORTED")

    # -------------------------------------------------------------- loss
    def _cos_detached(self, mats):
        """general_utils/metrics.py:342-381 (include_diag=False subtracts I; values only)."""
        if len(mats) <= 1:
            return None
        eye = torch.eye(mats[0].size(0), device=mats[0].device).unsqueeze(2)
        vs = [(g.detach() - eye).flatten().view(1, -1) for g in mats]
        vals = [float(Fn.cosine_similarity(vs[i], vs[j])) for i in range(len(vs)) for j in range(i + 1, len(vs))]
        return torch.tensor(vals, device=mats[0].device).view(1, -1)

    def compute_loss(self, conditioning_X, preds, targets, factor_scores, factor_labels, gc_est_mode,
                     embedder_pretrain_loss=False, factor_pretrain_loss=False):
        """...withStateSmoothing.py:624-731 (base class :620-686) with autograd."""
        m = self.m
        dev = preds.device
        gc = self.GC(gc_est_mode, X=conditioning_X, threshold=False, ignore_lag=True)
        gc_lagged = self.GC(gc_est_mode, X=conditioning_X, threshold=False, ignore_lag=False)
        forecast = m.FORECAST_COEFF * sum(Fn.mse_loss(preds[:, :, i], targets[:, :, i]) for i in range(m.num_series))
        factor = torch.zeros(1, device=dev)
        nsup = m.num_supervised_factors
        if factor_scores is not None and factor_scores[0] is not None and nsup > 0:
            Lm = m.Lmax
            factor_labels = factor_labels.to(dev)
            if factor_labels.dim() == 3 and factor_labels.size(2) > Lm:
                for y, yhat in zip([factor_labels[:, :, Lm + l] for l in range(factor_labels.size(2) - Lm)],
                                   factor_scores):
                    factor = factor + m.FACTOR_SCORE_COEFF * Fn.mse_loss(yhat[:, :nsup], y[:, :nsup])
            else:
                y = factor_labels[:, :, 0] if factor_labels.dim() == 3 else factor_labels
                yhat = factor_scores[0]
                for extra in factor_scores[1:]:
                    yhat = yhat + extra
                yhat = yhat / (1. * len(factor_scores))
                factor = factor + m.FACTOR_SCORE_COEFF * Fn.mse_loss(yhat[:, :nsup], y[:, :nsup])
        fw_l1 = m.FACTOR_WEIGHT_L1_COEFF * (torch.norm(factor_scores[0], 1) - 1.)
        smooth = torch.zeros(1, device=dev)
        if m._WITH_SMOOTHING:
            eps = m.STATE_SCORE_SMOOTHING_EPSILON
            if m.num_sims == 2:
                d = factor_scores[0] - factor_scores[1]
                d = d * (d > eps)
                smooth = torch.sum(d ** 2.)
            elif m.num_sims > 2:
                for idx, (s0, s1, s2) in enumerate(zip(factor_scores[:-2], factor_scores[1:-1], factor_scores[2:])):
                    full = s2 - s0
                    d21 = s2 - s1
                    smooth = smooth + torch.sum((d21 * torch.gt(torch.abs(d21), torch.abs(full))) ** 2.)
                    if idx == 0:
                        d10 = s1 - s0
                        smooth = smooth + torch.sum((d10 * torch.gt(torch.abs(d10), torch.abs(full))) ** 2.)
            smooth = smooth * m.FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF
        cos_pen, adj = None, None
        for b in range(len(gc)):
            if len(gc[b]) > 1:
                v = m.FACTOR_COS_SIM_COEFF * torch.sum(self._cos_detached(gc[b]))
                cos_pen = v if cos_pen is None else cos_pen + v
            for G in gc_lagged[b]:
                v = m.ADJ_L1_REG_COEFF * sum(math.log(i + 2.) * torch.sum(torch.abs(G[:, :, i]))
                                             for i in range(G.size(2)))
                adj = v if adj is None else adj + v
        sm = smooth if m._WITH_SMOOTHING else 0.0
        if embedder_pretrain_loss:
            combo = factor + fw_l1 + sm
        elif factor_pretrain_loss:
            combo = forecast + fw_l1 + sm + adj
            if cos_pen is not None:
                combo = combo + cos_pen
        else:
            combo = forecast + factor + fw_l1 + sm + adj
            if cos_pen is not None:
                combo = combo + cos_pen
        terms = [forecast, factor, cos_pen, fw_l1]
        if m._WITH_SMOOTHING:
            terms.append(smooth)
        return combo, terms + [adj, None]

    # -------------------------------------------------------------- training
    def step_loss(self, X, Y, output_length, **flags):
        m = self.m
        Lm = m.Lmax
        x_sims, _, _, labels = self.forward(X[:, :Lm, :])
        tgt = X[:, Lm:Lm + m.num_sims * output_length, :]
        return self.compute_loss(X[:, :m.embed_lag, :], x_sims, tgt, labels, Y, m.primary_gc_est_mode, **flags), labels

    def batch_update(self, kinds, X, Y, optimizerA, optimizerB, output_length, confusion=None):
        """One batch_update (...withStateSmoothing.py:734-933) for the update kinds of its phase."""
        m = self.m
        emb = m.factor_score_embedder
        labels = None
        for kind in kinds:
            if kind == "pretrain_embedder":
                emb.train()
                optimizerA.zero_grad()
                (loss, _), labels = self.step_loss(X, Y, output_length, embedder_pretrain_loss=True)
                loss.backward()
                self._step(optimizerA)
            elif kind in ("pretrain_factor", "acclimate", "post_train"):
                emb.eval()
                optimizerB.zero_grad()
                (loss, _), labels = self.step_loss(X, Y, output_length, factor_pretrain_loss=True)
                loss.backward()
                self._step(optimizerB)
            elif kind == "combined":
                emb.train()
                optimizerA.zero_grad()
                optimizerB.zero_grad()
                (loss, _), labels = self.step_loss(X, Y, output_length)
                loss.backward()
                self._step(optimizerA)
                self._step(optimizerB)
        if confusion is not None and labels is not None and m.num_supervised_factors > 0 and kinds and \
                kinds[-1] in ("pretrain_embedder", "combined"):
            n = m.num_supervised_factors
            lab = Y[:, :n, m.Lmax] if (Y.dim() == 3 and Y.size(2) > m.Lmax) else (Y[:, :n, 0] if Y.dim() == 3 else Y[:, :n])
            pred = labels[0][:, :n].detach().argmax(1).cpu().numpy()
            true = lab.argmax(1).cpu().numpy()
            for t_, p_ in zip(true, pred):
                confusion[t_, p_] += 1
        return confusion

    @torch.no_grad()
    def validate(self, batches, output_length=1):
        """validate_training averages (:1650-1790): forecast, factor, cos, fw_l1, smooth, adj, combo."""
        m = self.m
        m.factor_score_embedder.eval()
        dev = m.factors[0].networks[0].layers[0].weight.device
        keys = ["forecast", "factor", "cos", "fw_l1", "smooth", "adj", "combo"]
        coeff = {"forecast": m.FORECAST_COEFF, "factor": m.FACTOR_SCORE_COEFF, "cos": m.FACTOR_COS_SIM_COEFF,
                 "fw_l1": m.FACTOR_WEIGHT_L1_COEFF, "adj": m.ADJ_L1_REG_COEFF,
                 "smooth": getattr(m, "FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF", 0.0)}
        acc = dict((k, 0.0) for k in keys)
        cm = np.zeros((max(m.num_supervised_factors, 1),) * 2)
        for X, Y in batches:
            X, Y = X.to(dev, torch.float32), Y.to(dev, torch.float32)
            (combo, t), labels = self.step_loss(X, Y, output_length)
            if not m._WITH_SMOOTHING:
                t = t[:4] + [torch.zeros(1, device=dev)] + t[4:]
            for k, v in zip(keys[:6], t[:6]):
                v = 0.0 if v is None else float(v)
                acc[k] += v / coeff[k] if coeff[k] > 0 else v
            acc["combo"] += float(combo)
            n = m.num_supervised_factors
            if n > 0:
                lab = Y[:, :n, m.Lmax] if (Y.dim() == 3 and Y.size(2) > m.Lmax) else (Y[:, :n, 0] if Y.dim() == 3 else Y[:, :n])
                for t_, p_ in zip(lab.argmax(1).cpu().numpy(), labels[0][:, :n].argmax(1).cpu().numpy()):
                    cm[t_, p_] += 1
        nb = max(len(batches), 1)
        return dict((k, v / nb) for k, v in acc.items()), cm
