"""Device state of a REDCLIFF-S fit and the fused gfx950 training step.

``FitEngine`` owns, per model:
  * the packed parameter buffers (embedder group A, factor group B).  Every nn.Parameter
    of the model is re-pointed to a view of these buffers, so ``state_dict()``, the
    user's optimizers and the kernels all see the same memory;
  * the Adam moments of optimizerA / optimizerB, also exposed to the torch optimizers as
    views (``optimizer.state[p]['exp_avg']`` ...), with a shared step counter;
  * the workspace of the kernel chain and the device-resident copy of the training set
    (the reference re-reads and re-unpickles its data for every item,
    data/synthetic_datasets.py:135-244; here the windows are uploaded once).

One ``batch_update`` of the reference (models/redcliff_s_cmlp_withStateSmoothing.py:734-933)
is one ``redcliff_train_step`` call; an epoch is one ``redcliff_train_steps`` call.
"""
import ctypes

import numpy as np
import torch

from . import _native as nat
from .dgcnn import M1
from .kernels import factor_views, ptr

BMAX_LIMIT = 512  # windows per launch (include/redcliff_hip.h: Bmax <= 512)


# ----------------------------------------------------------------------------- phases
def phase_of_epoch(model, epoch_num):
    """...withStateSmoothing.py:741-759 -> list of update kinds run in this batch_update."""
    mode = model.training_mode
    if epoch_num <= model.num_pretrain_epochs - 1:
        kinds = []
        if "pretrain_embedder" in mode:
            kinds.append("pretrain_embedder")
        if "pretrain_factor" in mode:
            kinds.append("pretrain_factor")
        return kinds
    if "acclimate_factors" in mode and epoch_num <= model.num_pretrain_epochs + model.num_acclimation_epochs - 1:
        return ["acclimate"]
    if "combined" in mode:
        return ["combined"]
    if "post_train_factor" in mode:
        return ["post_train"]
    raise NotImplementedError()


def step_flags(model, kind, nsup):
    """flags_for, less optimizerB when the model's factors were replaced by a prior model's
    (initialize_factors_with_prior: the reference's optimizerB keeps the replaced parameters, so
    the loaded factors are never stepped).  flags 0: nothing of the update changes any state."""
    flags, nbn = flags_for(kind, nsup)
    if model.__dict__.get("_factors_detached", False):
        flags &= ~nat.STEP_B
        if not flags & nat.STEP_A:
            return 0, 0
    return flags, nbn


def flags_for(kind, nsup):
    """Loss terms / optimizer steps of one update kind (compute_loss flags, :718-729)."""
    conf = nat.CONFUSION if nsup > 0 else 0
    if kind == "pretrain_embedder":  # embedder_pretrain_loss: factor + fw_l1 (+ smoothing); optimizerA
        return nat.BN_TRAIN | nat.LOSS_FACTOR | nat.LOSS_FWL1 | nat.STEP_A | conf, 3
    if kind in ("pretrain_factor", "acclimate", "post_train"):  # factor_pretrain_loss; embedder eval; optimizerB
        return nat.LOSS_FORECAST | nat.LOSS_FWL1 | nat.LOSS_ADJ | nat.STEP_B, 0
    if kind == "combined":
        return (nat.BN_TRAIN | nat.LOSS_FORECAST | nat.LOSS_FACTOR | nat.LOSS_FWL1 | nat.LOSS_ADJ | nat.STEP_A |
                nat.STEP_B | conf), 3
    raise ValueError(kind)


def select_labels(Y, K, Lmax):
    """Label matrix (B, K) that compute_loss compares against (:635-661)."""
    Y = Y.to(torch.float32)
    if Y.dim() == 3:
        lab = Y[:, :, Lmax] if Y.size(2) > Lmax else Y[:, :, 0]
    elif Y.dim() == 2:
        lab = Y
    else:
        raise NotImplementedError("Cannot handle ground-truth labels with Y.size() == " + str(tuple(Y.size())))
    if lab.size(1) < K:
        lab = torch.cat([lab, torch.zeros(lab.size(0), K - lab.size(1), dtype=lab.dtype, device=lab.device)], 1)
    return lab[:, :K].contiguous()


# ----------------------------------------------------------------------------- engine
class FitEngine:
    def __init__(self, model):
        self.model = model
        emb = model.factor_score_embedder
        self.dgcnn = emb.dgcnn.dgcnn
        self.p = model.num_series
        self.L = model.gen_lag
        self.K = model.num_factors_nK
        self.nsup = model.num_supervised_factors
        self.h = model.gen_hidden[0]
        self.F = self.dgcnn.in_channels
        self.n = self.dgcnn.num_layers
        self.H = self.dgcnn.hid_channels
        self.Lmax = max(model.gen_lag, model.embed_lag)
        self.device = self.dgcnn.A.device
        self.sig = bool(emb.use_sigmoid_restriction)
        self.ecc = float(emb.sigmoid_eccentricity_coeff or 0.0)
        self._emb_layout()
        PA = self.eo["total"]
        PB = self.fo["total"]
        dev = self.device
        self.emb = torch.empty(PA, device=dev, dtype=torch.float32)
        self.fac = torch.empty(PB, device=dev, dtype=torch.float32)
        self.bn = torch.empty(2, self.F, device=dev, dtype=torch.float32)
        self.acc = torch.zeros(8, device=dev, dtype=torch.float64)
        self.conf = torch.zeros(max(self.nsup, 1) ** 2, device=dev, dtype=torch.int32)
        self.opt = {"A": None, "B": None}  # bound optimizer state per group
        self.ws = None
        self.ws_dims = None
        self.hyper_key = None
        self.hyper_dev = None
        self.supports_fresh = False
        self._a_version = -1
        self.dataset_cache = {}
        self.pack = None  # ReplicaPack this fit belongs to (redcliff_amd.replicas), if any
        self.pack_index = None
        self.bind()

    # ------------------------------------------------------------------ layout / binding
    def _emb_layout(self):
        p, n, F, H, K = self.p, self.n, self.F, self.H, self.K
        o = {"A": 0}
        o["gcW"] = o["A"] + p * p
        o["bnw"] = o["gcW"] + n * F * H
        o["bnb"] = o["bnw"] + F
        o["fc1W"] = o["bnb"] + F
        o["fc1b"] = o["fc1W"] + M1 * p * H
        o["fc2W"] = o["fc1b"] + M1
        o["fc2b"] = o["fc2W"] + K * M1
        o["total"] = o["fc2b"] + K
        self.eo = o
        kp = K * self.p
        fo = {"W0": 0}
        fo["b0"] = fo["W0"] + kp * self.h * self.p * self.L
        fo["W1"] = fo["b0"] + kp * self.h
        fo["b1"] = fo["W1"] + kp * self.h
        fo["total"] = fo["b1"] + kp
        self.fo = fo

    def _emb_pairs(self):
        g, o, E = self.dgcnn, self.eo, self.emb
        p, n, F, H, K = self.p, self.n, self.F, self.H, self.K
        pairs = [(g.A, E[o["A"]:o["A"] + p * p].view(p, p))]
        for i in range(n):
            pairs.append((g.layer1.gc1[i].weight, E[o["gcW"] + i * F * H:o["gcW"] + (i + 1) * F * H].view(F, H)))
        pairs += [(g.BN1.weight, E[o["bnw"]:o["bnw"] + F]), (g.BN1.bias, E[o["bnb"]:o["bnb"] + F]),
                  (g.fc1.linear.weight, E[o["fc1W"]:o["fc1W"] + M1 * p * H].view(M1, p * H)),
                  (g.fc1.linear.bias, E[o["fc1b"]:o["fc1b"] + M1]),
                  (g.fc2.linear.weight, E[o["fc2W"]:o["fc2W"] + K * M1].view(K, M1)),
                  (g.fc2.linear.bias, E[o["fc2b"]:o["fc2b"] + K])]
        return pairs

    def _fac_pairs(self):
        return factor_views(self.fac, list(self.model.factors), self.p, self.h, self.L)

    def bind(self, copy=True):
        """Copy current parameter values into the packed buffers and alias the parameters.
        copy=False: the buffers already hold the values (attach_pack moved them in bulk)."""
        with torch.no_grad():
            self.pairs = self._emb_pairs() + self._fac_pairs()
            if copy:  # one multi-tensor launch instead of a copy kernel per parameter
                views = [view for _, view in self.pairs]
                srcs = [prm.detach().to(view.device).reshape(view.shape) for prm, view in self.pairs]
                torch._foreach_copy_(views, srcs)
            for prm, view in self.pairs:
                prm.data = view
            bnm = self.dgcnn.BN1
            self.bn[0].copy_(bnm.running_mean)
            self.bn[1].copy_(bnm.running_var)
            bnm.running_mean = self.bn[0]
            bnm.running_var = self.bn[1]
        self.bound_ptrs = [prm.data_ptr() for prm, _ in self.pairs]
        self.supports_fresh = False

    def ensure_bound(self):
        cur = [prm.data_ptr() for prm, _ in self.pairs]
        bn = self.dgcnn.BN1
        if (cur != self.bound_ptrs or bn.running_mean.data_ptr() != self.bn[0].data_ptr()
                or bn.running_var.data_ptr() != self.bn[1].data_ptr()):
            self.bind()
            for g in ("A", "B"):
                if self.opt[g] is not None:
                    self._attach_state(g)

    def invalidate(self):
        """Parameters were modified in place from outside: supports must be recomputed."""
        self.supports_fresh = False

    # ------------------------------------------------------------------ optimizers
    def _group_params(self, g):
        n_emb = 1 + self.n + 6
        pr = [prm for prm, _ in self.pairs]
        return pr[:n_emb] if g == "A" else pr[n_emb:]

    def _attach_state(self, g):
        st = self.opt[g]
        opt = st["opt"]
        mflat, vflat = st["m"], st["v"]
        base = self.emb if g == "A" else self.fac
        for prm in self._group_params(g):
            off = (prm.data_ptr() - base.data_ptr()) // 4
            n = prm.numel()
            opt.state[prm] = {"step": st["step"], "exp_avg": mflat[off:off + n].view_as(prm),
                              "exp_avg_sq": vflat[off:off + n].view_as(prm)}

    def bind_optimizer(self, g, opt):
        st = self.opt[g]
        if st is not None and st["opt"] is opt:
            return st
        if not isinstance(opt, torch.optim.Adam):
            raise NotImplementedError("the fused step implements torch.optim.Adam (model_utils.py:747-762)")
        if len(opt.param_groups) != 1:
            raise NotImplementedError("one parameter group per optimizer expected")
        grp = opt.param_groups[0]
        if grp.get("amsgrad") or grp.get("maximize") or grp.get("decoupled_weight_decay", False):
            raise NotImplementedError("amsgrad / maximize / decoupled weight decay are not used by REDCLIFF-S")
        mine = set(id(x) for x in self._group_params(g))
        theirs = set(id(x) for x in grp["params"])
        if mine != theirs:
            raise ValueError("optimizer%s must own exactly model.gen_model[%d].parameters()" % (g, 0 if g == "A" else 1))
        base = self.emb if g == "A" else self.fac
        m, v = self._new_moments(g)
        step = 0
        for prm in self._group_params(g):
            s = opt.state.get(prm)
            if s and "exp_avg" in s:  # resume from a torch-stepped optimizer
                off = (prm.data_ptr() - base.data_ptr()) // 4
                m[off:off + prm.numel()] = s["exp_avg"].reshape(-1)
                v[off:off + prm.numel()] = s["exp_avg_sq"].reshape(-1)
                step = int(float(s["step"]))
        st = {"opt": opt, "m": m, "v": v, "t": step, "step": torch.tensor(float(step), dtype=torch.float32)}
        self.opt[g] = st
        self._attach_state(g)
        return st

    def _new_moments(self, g):
        """Zeroed Adam moment buffers of group g: rows of the replica pack when packed."""
        if self.pack is not None:
            m, v = self.pack.moments(g, self.pack_index)
            m.zero_()
            v.zero_()
            return m, v
        base = self.emb if g == "A" else self.fac
        return torch.zeros_like(base), torch.zeros_like(base)

    def attach_pack(self, pack, index):
        """Move this fit's parameters, BatchNorm buffers and Adam moments into row `index`
        of a ReplicaPack (packed [R][...] buffers, one launch for R fits).  The module's
        parameters and the optimizers' state stay views, now of the pack's rows."""
        self.ensure_bound()
        emb_old, fac_old, bn_old = self.emb, self.fac, self.bn
        self.pack, self.pack_index = pack, index
        self.emb, self.fac, self.bn = pack.emb[index], pack.fac[index], pack.bn[:, index]
        with torch.no_grad():
            self.emb.copy_(emb_old)
            self.fac.copy_(fac_old)
            self.bn.copy_(bn_old)
        self.bind(copy=False)
        for g in ("A", "B"):
            st = self.opt[g]
            if st is None:
                continue
            m, v = pack.moments(g, index)
            with torch.no_grad():
                m.copy_(st["m"])
                v.copy_(st["v"])
            st["m"], st["v"] = m, v
            self._attach_state(g)

    def _sync_steps(self):
        for g in ("A", "B"):
            st = self.opt[g]
            if st is not None:
                st["step"].fill_(float(st["t"]))

    # ------------------------------------------------------------------ hyper-parameters
    def _hyper(self):
        m = self.model
        bnm = self.dgcnn.BN1
        gA = self.opt["A"]["opt"].param_groups[0] if self.opt["A"] else None
        gB = self.opt["B"]["opt"].param_groups[0] if self.opt["B"] else None

        def adam(gr):
            if gr is None:
                return (0.0, (0.9, 0.999), 1e-8, 0.0)
            return (float(gr["lr"]), tuple(float(b) for b in gr["betas"]), float(gr["eps"]), float(gr["weight_decay"]))

        key = (m.FORECAST_COEFF, m.FACTOR_SCORE_COEFF, m.FACTOR_COS_SIM_COEFF, m.FACTOR_WEIGHT_L1_COEFF,
               getattr(m, "FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF", 0.0), m.ADJ_L1_REG_COEFF, float(bnm.eps),
               float(bnm.momentum if bnm.momentum is not None else 0.1), adam(gA), adam(gB))
        if key != self.hyper_key:
            h = nat.ReplicaHyper()
            (h.c_forecast, h.c_factor, h.c_cos, h.c_fwl1, h.c_smooth, h.c_adj) = [float(x) for x in key[:6]]
            h.bn_eps, h.bn_momentum = key[6], key[7]
            h.A = nat.adam_hyper(key[8][0], key[8][1], key[8][2], key[8][3])
            h.B = nat.adam_hyper(key[9][0], key[9][1], key[9][2], key[9][3])
            raw = np.frombuffer(bytes(h), dtype=np.uint8).copy()
            self.hyper_dev = torch.from_numpy(raw).to(self.device)
            self.hyper_key = key
        return self.hyper_dev

    # ------------------------------------------------------------------ workspace
    def dims(self, Bmax, T):
        return nat.Dims(R=1, Bmax=int(Bmax), T=int(T), p=self.p, L=self.L, K=self.K, h=self.h, F=self.F, n=self.n,
                        H=self.H, M1=M1, nsup=self.nsup, use_sigmoid=int(self.sig), sigmoid_ecc=self.ecc)

    def status_view(self):
        """int32 device view of this engine's workspace status word (WsOff.errw; see
        _native.raise_on_status)."""
        return nat.status_view(self.ws, self.ws_off, 1)

    def raise_on_status(self, words, where):
        nat.raise_on_status(words, self.status_view(), where)

    def check_device_status(self, where="check"):
        """Read the status word (synchronises) and raise if a merged-backward hand-off timed out
        since the last check.  fit() checks once per epoch inside its single copy back,
        validate_training after its copy back; callers driving batch_update themselves can
        call model.check_device_status()."""
        if self.ws is not None:
            self.raise_on_status(self.status_view().cpu().numpy(), where)

    def workspace(self, Bmax, T):
        Bmax = max(int(Bmax), 1)
        if self.ws_dims is not None and self.ws_dims[0] >= Bmax:
            d = self.dims(self.ws_dims[0], T)
        else:
            self.check_device_status("workspace growth")  # the old workspace's word would be lost
            d = self.dims(Bmax, T)
            nbytes = nat.lib().redcliff_workspace_bytes(ctypes.byref(d))
            if nbytes == 0:
                nat.check(-1, "workspace_bytes")
            self.ws = torch.zeros(nbytes // 4, device=self.device, dtype=torch.float32)
            self.ws_dims = (Bmax,)
            self.ws_off = nat.workspace_layout(d)
            self.supports_fresh = False
        return d

    # ------------------------------------------------------------------ data
    def bn_stats(self, d, X, N, B):
        nb = (N + B - 1) // B
        st = torch.empty(nb, 2, self.F, device=self.device, dtype=torch.float64)
        nat.check(nat.lib().redcliff_bn_batch_stats(ctypes.byref(d), ptr(X), 0, int(N), int(B), ptr(st), 0,
                                                    _stream()), "bn_batch_stats")
        return st

    def stage(self, X, Y):
        """One host batch -> device tensors (X (B,T,p), labels (B,K), BN batch stats)."""
        X = X.to(self.device, torch.float32).contiguous()
        B, T, p = X.shape
        if p != self.p:
            raise ValueError("expected %d channels, got %d" % (self.p, p))
        lab = select_labels(Y.to(self.device), self.K, self.Lmax) if Y is not None else None
        d = self.workspace(B, T)
        st = self.bn_stats(d, X, B, B)
        return X, lab, st, d

    def cache_dataset(self, loader):
        """Upload an iterable of (X, Y) batches once; later epochs replay the same order
        (the reference DataLoader has no shuffling: data/synthetic_datasets.py:272-276)."""
        key = id(loader)
        if key in self.dataset_cache:
            return self.dataset_cache[key]
        xs, ys, sizes = [], [], []
        for X, Y in loader:
            xs.append(X.to(torch.float32))
            ys.append(select_labels(Y, self.K, self.Lmax) if Y is not None else torch.zeros(X.shape[0], self.K))
            sizes.append(int(X.shape[0]))
        Xall = torch.cat(xs, 0).to(self.device).contiguous()
        lab = torch.cat(ys, 0).to(self.device, torch.float32).contiguous()
        rows = np.cumsum([0] + sizes[:-1]).astype(np.int64)
        # the BatchNorm statistics kernel takes any batch size; the step workspace is sized for
        # the batches (a data-parallel fit's global batches may exceed one launch's Bmax: it
        # sizes the workspace for its shards itself)
        d = self.workspace(max(sizes), Xall.shape[1]) if max(sizes) <= BMAX_LIMIT else self.dims(1, Xall.shape[1])
        if all(s == sizes[0] for s in sizes[:-1]) and sizes[-1] <= sizes[0]:
            # consecutive equal batches (a ragged last one allowed): one launch for all of them
            stats = self.bn_stats(d, Xall, int(Xall.shape[0]), sizes[0])
        else:
            stats = torch.cat([self.bn_stats(d, Xall[r:r + s], s, s) for r, s in zip(rows, sizes)], 0)
        ds = {"X": Xall, "lab": lab, "rows": rows, "sizes": np.asarray(sizes, dtype=np.int32),
              "stats": stats.contiguous(), "T": int(Xall.shape[1]), "Bmax": max(sizes),
              "len": len(sizes), "loader": loader}
        self.dataset_cache[key] = ds
        return ds

    # ------------------------------------------------------------------ step launch
    def _fresh_state(self):
        """Pick up changes made outside the kernels: an optimizer stepped by torch (its shared
        step tensor moved) and an adjacency A modified by a torch op (A's version counter, shared
        with the packed buffer it views, moved) -- the supports must then be rebuilt."""
        for g in ("A", "B"):
            st = self.opt[g]
            if st is not None:
                tv = int(float(st["step"]))
                if tv != st["t"]:
                    st["t"] = tv
        if self.supports_fresh and self.dgcnn.A._version != self._a_version:
            self.supports_fresh = False

    def _args(self, d, flags, nbn, X, lab, stats):
        self._fresh_state()
        a = nat.StepArgs()
        a.d = d
        a.flags = flags | (0 if self.supports_fresh else nat.REFRESH_SUPPORTS)
        a.n_bn_updates = nbn
        stA, stB = self.opt["A"], self.opt["B"]
        a.tA = (stA["t"] + 1) if stA else 1
        a.tB = (stB["t"] + 1) if stB else 1
        a.X = X.data_ptr()
        a.labels = lab.data_ptr() if lab is not None else None
        a.bn_stats = stats.data_ptr() if stats is not None else None
        a.emb, a.emb_stride = self.emb.data_ptr(), self.emb.numel()
        a.fac, a.fac_stride = self.fac.data_ptr(), self.fac.numel()
        if stA:
            a.emb_m, a.emb_v = stA["m"].data_ptr(), stA["v"].data_ptr()
        else:
            a.emb_m = a.emb_v = self.emb.data_ptr()
        if stB:
            a.fac_m, a.fac_v = stB["m"].data_ptr(), stB["v"].data_ptr()
        else:
            a.fac_m = a.fac_v = self.fac.data_ptr()
        a.bn_rm, a.bn_rv = self.bn[0].data_ptr(), self.bn[1].data_ptr()
        a.hyper = self._hyper().data_ptr()
        a.ws, a.ws_bytes = self.ws.data_ptr(), self.ws.numel() * 4
        a.acc = self.acc.data_ptr()
        a.confusion = self.conf.data_ptr()
        return a

    def _mark_fresh(self):
        self.supports_fresh = True
        self._a_version = self.dgcnn.A._version

    def _after(self, flags, nbn, nsteps, bn=True):
        self._mark_fresh()
        if flags & nat.STEP_A:
            self.opt["A"]["t"] += nsteps
        if flags & nat.STEP_B:
            self.opt["B"]["t"] += nsteps
        if nbn and bn:  # (a ReplicaPack advances its replicas' counters in one add)
            self.dgcnn.BN1.num_batches_tracked.add_(nbn * nsteps)
        self._sync_steps()

    def run_steps(self, kinds, X, lab, stats, d, rows, sizes, oA, oB):
        """Run the update kinds of one phase over consecutive batches (rows/sizes)."""
        self.ensure_bound()
        for kind in kinds:
            flags, nbn = step_flags(self.model, kind, self.nsup)
            if flags == 0:
                continue
            if flags & nat.STEP_A:
                self.bind_optimizer("A", oA)
            if flags & nat.STEP_B:
                self.bind_optimizer("B", oB)
            if not (flags & nat.BN_TRAIN):
                stats_p = None
            else:
                stats_p = stats
            a = self._args(d, flags, nbn, X, lab, stats_p)
            rows_a = np.ascontiguousarray(rows, dtype=np.int64)
            sizes_a = np.ascontiguousarray(sizes, dtype=np.int32)
            nat.check(nat.lib().redcliff_train_steps(ctypes.byref(a), len(rows_a), rows_a.ctypes.data_as(ctypes.c_void_p),
                                                     sizes_a.ctypes.data_as(ctypes.c_void_p), 2 * self.F, _stream()),
                      "train_steps")
            self._after(flags, nbn, len(rows_a))

    def plan_steps(self, kind, X, lab, stats, d, rows, sizes, oA, oB):
        """A prepared epoch of one update kind: the argument block, batch order and statistics
        are built once; ``StepPlan.run()`` launches the epoch with only the Adam step numbers
        refreshed (the host cost of one epoch is one C call)."""
        return StepPlan(self, kind, X, lab, stats, d, rows, sizes, oA, oB)

    VAL_GROUP = 7  # validation batches per replicated launch (R < 8 keeps the single fit's kernel paths)

    def run_values(self, X, lab, d, rows, sizes, train_bn=False, stats=None, confusion=True, grouped=True, host=True):
        """validate_training body over consecutive batches; returns (acc[8], confusion).
        grouped=False: one launch chain per batch (the reference's loop, used by the tests).
        host=False (eval mode): the per-batch device rows (acc [nb][8], confusion [nb][ns*ns]),
        still on the device -- finish with values_from_rows after copying them back."""
        self.ensure_bound()
        flags = nat.VALUES | (nat.CONFUSION if (confusion and self.nsup > 0) else 0)
        rows = np.asarray(rows, dtype=np.int64)
        sizes = np.asarray(sizes, dtype=np.int32)
        if not host:
            assert not train_bn
            return self._run_values_grouped(X, lab, d, rows, sizes, flags, host=False)
        if grouped and not train_bn and len(sizes) > 1:
            return self._run_values_grouped(X, lab, d, rows, sizes, flags)
        self.acc.zero_()
        self.conf.zero_()
        if train_bn:
            flags |= nat.BN_TRAIN
        a = self._args(d, flags, 0, X, lab, stats if train_bn else None)
        rows_a = np.ascontiguousarray(rows, dtype=np.int64)
        sizes_a = np.ascontiguousarray(sizes, dtype=np.int32)
        nat.check(nat.lib().redcliff_train_steps(ctypes.byref(a), len(rows_a), rows_a.ctypes.data_as(ctypes.c_void_p),
                                                 sizes_a.ctypes.data_as(ctypes.c_void_p), 2 * self.F, _stream()),
                  "validate")
        self._mark_fresh()
        return self.acc.cpu().numpy(), self.conf.cpu().numpy().reshape(max(self.nsup, 1), max(self.nsup, 1))

    def values_from_rows(self, accs, confs):
        """(acc[8], confusion) of validate_training from the per-batch rows of run_values(host=False)
        (host arrays): the batch loop's running sum, left to right in batch order."""
        ns = max(self.nsup, 1)
        return (np.cumsum(np.asarray(accs, dtype=np.float64), axis=0)[-1],
                np.asarray(confs).reshape(-1, ns, ns).sum(axis=0).astype(np.int32))

    def _run_values_grouped(self, X, lab, d, rows, sizes, flags, host=True):
        """Eval-mode validation with the batches on the replica axis: a run of g <= VAL_GROUP
        consecutive equal-size batches is ONE launch chain of g "replicas" that all read this
        fit's parameters (parameter strides 0, window / label strides one batch) instead of g
        dependent chains (validation updates nothing, so the batches are independent), and all
        chains are enqueued before the one copy back.  Each batch's values land in its own
        accumulator row as 0 + v (the batch loop adds v to the running sum); the rows are then
        summed left to right in batch order, so the totals are bit-identical to the loop."""
        ns = max(self.nsup, 1)
        nb = len(sizes)
        gmax = min(self.VAL_GROUP, nb)
        dg = nat.Dims(**dict((f, getattr(d, f)) for f, _ in nat.Dims._fields_))
        dg.R = gmax
        key = (gmax, nb, d.Bmax, d.T)
        vr = getattr(self, "_val_rep", None)
        if vr is None or vr["key"] != key:
            nbytes = nat.lib().redcliff_workspace_bytes(ctypes.byref(dg))
            if nbytes == 0:
                nat.check(-1, "workspace_bytes")
            vr = {"key": key, "ws": torch.zeros(nbytes // 4, device=self.device, dtype=torch.float32),
                  "acc": torch.zeros(nb, 8, device=self.device, dtype=torch.float64),
                  "conf": torch.zeros(nb, ns * ns, device=self.device, dtype=torch.int32)}
            self._val_rep = vr
        rm = self.bn[0].unsqueeze(0).expand(gmax, self.F).contiguous()
        rv = self.bn[1].unsqueeze(0).expand(gmax, self.F).contiguous()
        hg = self._hyper().repeat(gmax)
        vr["acc"].zero_()
        vr["conf"].zero_()
        a = self._args(dg, flags | nat.REFRESH_SUPPORTS, 0, X, lab, None)
        a.emb_stride, a.fac_stride = 0, 0  # every "replica" reads this fit's parameters
        a.bn_rm, a.bn_rv = rm.data_ptr(), rv.data_ptr()
        a.hyper = hg.data_ptr()
        a.ws, a.ws_bytes = vr["ws"].data_ptr(), vr["ws"].numel() * 4
        i = 0
        while i < nb:
            g = 1
            while (g < gmax and i + g < nb and sizes[i + g] == sizes[i]
                   and rows[i + g] == rows[i] + g * int(sizes[i])):
                g += 1
            B = int(sizes[i])
            a.d.R = g
            a.B, a.row0 = B, int(rows[i])
            a.x_rstride = B * d.T * self.p  # replica r = batch i + r
            a.lab_rstride = B * self.K
            a.acc = vr["acc"][i].data_ptr()
            a.confusion = vr["conf"][i].data_ptr()
            nat.check(nat.lib().redcliff_train_step(ctypes.byref(a), _stream()), "validate (replicated batches)")
            i += g
        if not host:
            return vr["acc"], vr["conf"]
        return self.values_from_rows(vr["acc"].cpu().numpy(), vr["conf"].cpu().numpy())

    def forward_outputs(self, X, train_bn, bn_updates):
        """Embedder + factors + mixing on windows X (B, T>=Lmax, p): returns w_raw, y, xsim."""
        self.ensure_bound()
        X = X.to(self.device, torch.float32).contiguous()
        B, T, _ = X.shape
        d = self.workspace(B, T)
        stats = self.bn_stats(d, X, B, B) if train_bn else None
        flags = nat.STORE_OUTPUTS | (nat.BN_TRAIN if train_bn else 0)
        a = self._args(d, flags, bn_updates if train_bn else 0, X, None, stats)
        a.B = B
        a.row0 = 0
        nat.check(nat.lib().redcliff_train_step(ctypes.byref(a), _stream()), "forward")
        self._mark_fresh()
        if train_bn and bn_updates:
            self.dgcnn.BN1.num_batches_tracked.add_(bn_updates)
        o = self.ws_off
        w = self.ws[o["w"]:o["w"] + B * self.K].view(B, self.K).clone()
        y = torch.empty(B, self.K, self.p, device=self.device, dtype=torch.float32)
        nat.check(nat.lib().redcliff_step_predictions(ctypes.byref(d), B, ptr(self.ws), ptr(y), y.numel(), _stream()),
                  "step_predictions")
        xs = self.ws[o["xsim"]:o["xsim"] + B * self.p].view(B, self.p).clone()
        return w, y, xs

    def embed_raw(self, X):
        """Raw embedder outputs w (B, K) of windows X (B, T >= Lmax, p) with the BatchNorm running
        statistics (eval mode): the embedder launch alone (no factor networks, no step)."""
        self.ensure_bound()
        X = X.to(self.device, torch.float32).contiguous()
        B, T, _ = X.shape
        d = self.workspace(B, T)
        a = self._args(d, 0, 0, X, None, None)
        a.B = B
        a.row0 = 0
        nat.check(nat.lib().redcliff_train_step(ctypes.byref(a), _stream()), "embed")
        self._mark_fresh()
        o = self.ws_off
        return self.ws[o["w"]:o["w"] + B * self.K].view(B, self.K).clone()

    def gc_norms(self):
        """(G (K,p,p,L), G0 (K,p,p)) of the current factor weights."""
        self.ensure_bound()
        d = nat.Dims(R=1, Bmax=1, T=self.L, p=self.p, L=self.L, K=self.K, h=self.h, F=self.L, n=1, H=1, M1=1,
                     nsup=0, use_sigmoid=0, sigmoid_ecc=0.0)
        G = torch.empty(self.K, self.p, self.p, self.L, device=self.device, dtype=torch.float32)
        G0 = torch.empty(self.K, self.p, self.p, device=self.device, dtype=torch.float32)
        nat.check(nat.lib().redcliff_gc_norms(ctypes.byref(d), ptr(self.fac), self.fac.numel(), ptr(G), ptr(G0),
                                              _stream()), "gc_norms")
        return G, G0


class StepPlan:
    """One update kind over a fixed batch sequence (an epoch of fit(), or a bench run), with
    everything but the Adam step numbers resolved up front.  Valid while the model's
    parameters stay bound to this engine (fit loops and the bench do not rebind them)."""

    def __init__(self, eng, kind, X, lab, stats, d, rows, sizes, oA, oB):
        eng.ensure_bound()
        self.eng = eng
        self.flags, self.nbn = step_flags(eng.model, kind, eng.nsup)
        if self.flags & nat.STEP_A:
            eng.bind_optimizer("A", oA)
        if self.flags & nat.STEP_B:
            eng.bind_optimizer("B", oB)
        self.stats = stats.contiguous() if (stats is not None and self.flags & nat.BN_TRAIN) else None
        self.X, self.lab = X, lab  # keep the buffers alive
        self.a = eng._args(d, self.flags, self.nbn, X, lab, self.stats)
        self.rows = np.ascontiguousarray(rows, dtype=np.int64)
        self.sizes = np.ascontiguousarray(sizes, dtype=np.int32)
        self.n = len(self.rows)
        self._rows_p = self.rows.ctypes.data_as(ctypes.c_void_p)
        self._sizes_p = self.sizes.ctypes.data_as(ctypes.c_void_p)
        self._fn = nat.lib().redcliff_train_steps
        self._bn_step = 2 * eng.F

    def run(self):
        eng, a = self.eng, self.a
        if self.flags == 0:
            return
        eng._fresh_state()
        stA, stB = eng.opt["A"], eng.opt["B"]
        a.tA = (stA["t"] + 1) if stA else 1
        a.tB = (stB["t"] + 1) if stB else 1
        a.flags = self.flags | (0 if eng.supports_fresh else nat.REFRESH_SUPPORTS)
        if self.nbn:
            # BatchNorm's num_batches_tracked, which no kernel reads, advanced ahead of the chain (same
            # stream): its tiny launch runs while the host still enqueues the steps, not after them
            eng.dgcnn.BN1.num_batches_tracked.add_(self.nbn * self.n)
        rc = self._fn(ctypes.byref(a), self.n, self._rows_p, self._sizes_p, self._bn_step, _stream())
        if rc != 0:
            nat.check(rc, "train_steps (plan)")
        eng._after(self.flags, self.nbn, self.n, bn=False)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

