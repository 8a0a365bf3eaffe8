"""Grid-search replicas packed into one launch.

The reference runs one hyper-parameter combination per SLURM array task
(train/REDCLIFF_S_CMLP_tst100hzRerun1024AvgReg_gsSmooth1.py:125-160, 278-309): every task
builds its own model, reads the same dataset and fits independently.  On MI355X a single
fit at B=128 occupies a few hundred workgroups for a few microseconds per kernel, so R
fits with identical shapes are packed into ONE launch of the fused step: every kernel
carries the replica on blockIdx.y and every per-fit buffer (parameters, Adam moments,
BatchNorm running statistics, hyper-parameters, workspace, loss accumulators) is a row
of an [R][...] tensor.  Replicas may differ in everything that is not a shape: seeds,
coefficient dicts, learning rates / eps / weight decay of both optimizers, BatchNorm
momentum, stopping-criterion coefficients, the phase schedule (pretrain / acclimation epochs,
training mode: the TST grid varies them, train/REDCLIFF_S_CMLP_tst100hzRerun1024AvgReg_gsSmooth1.py:
297-298) and the data.  A grid whose points share one dataset (the TST grid) passes one loader;
a grid of one model over many datasets ("subjects": the synthetic grid is one model config over
990 dataset variants, train/REDCLIFF_S_CMLP_synSysInnovGauss1030_BSCgsSmooth3Parsim.py:66-72)
passes ``PerReplica`` loaders and true graphs, which become [R][N][T][p] device tensors read
through the kernels' replica strides.  Every epoch the active replicas are grouped by the update
kinds their schedules give that epoch and each group is one launch chain; a replica's Adam step
numbers ride in its hyper-parameter row (``t_offset``), so replicas that stepped a group
different numbers of times share launches.  ``grid_packs`` groups a grid by shape (and data
shape), ``shard_grid`` deals whole shape classes to GPUs.

``ReplicaPack.fit`` is the packed counterpart of ``fit()`` (...withStateSmoothing.py:
1175-1647): every replica keeps its own histories, GC-progress trackers, best-epoch
snapshot, checkpoints and early-stopping rule (redcliff_amd.fit_loop.FitTracker -- the very
code the single fit runs); a replica that stops leaves the launch's active list, so its
state freezes and its workgroups are no longer launched.

Each model stays a normal drop-in module: its parameters and its optimizers' state are
views of its pack row, so ``state_dict()``, ``GC()``, ``forward()`` and the single-fit
methods keep working on it between packed epochs.
"""
import ctypes
import gc
import os
import time

import numpy as np
import torch

from . import _native as nat
from . import metrics as M
from .engine import _stream, flags_for, phase_of_epoch
from .fit_loop import (DeferredHistories, FitTracker, ParamSnapshot, conditional_gc_estimates, confusion_rates_many,
                       gc_progress_many, restore_parameters, standalone_copy, train_confusion_many)


class PerReplica(list):
    """Marks a per-replica argument of ``ReplicaPack.fit`` / ``cache_dataset``: element r belongs
    to replica r -- its own training or validation loader (a subject / dataset of the grid; every
    replica's loader must yield the same batch sizes) or its own list of true graphs."""


class ReplicaPack:
    """R REDCLIFF-S fits with identical shapes stepped together.

    models: list of REDCLIFF_S_CMLP[_withStateSmoothing] on one GPU; optimizers: list of
    (optimizerA, optimizerB) per model (torch.optim.Adam over gen_model[0] / gen_model[1],
    general_utils/model_utils.py:747-762)."""

    def __init__(self, models, optimizers):
        if not models:
            raise ValueError("empty replica pack")
        if len(optimizers) != len(models):
            raise ValueError("one (optimizerA, optimizerB) pair per model")
        self.models = list(models)
        self.optimizers = [tuple(o) for o in optimizers]
        self.engines = [m.engine() for m in self.models]
        e0 = self.engines[0]
        shape = self._shape(e0)
        for e in self.engines[1:]:
            if self._shape(e) != shape:
                raise ValueError("replicas must share every shape (p, L, K, nsup, h, F, n, H, sigmoid): %s vs %s"
                                 % (self._shape(e), shape))
            if e.device != e0.device:
                raise ValueError("replicas must live on one device")
        self.R = R = len(self.models)
        self.device = e0.device
        PA, PB, F = e0.emb.numel(), e0.fac.numel(), e0.F
        dev = self.device
        self.emb = torch.empty(R, PA, device=dev, dtype=torch.float32)
        self.fac = torch.empty(R, PB, device=dev, dtype=torch.float32)
        self.m = {"A": torch.zeros(R, PA, device=dev), "B": torch.zeros(R, PB, device=dev)}
        self.v = {"A": torch.zeros(R, PA, device=dev), "B": torch.zeros(R, PB, device=dev)}
        # [2][R][F]: the kernels read running_mean[r*F + f] / running_var[r*F + f]
        self.bn = torch.empty(2, R, F, device=dev, dtype=torch.float32)
        self.acc = torch.zeros(R, 8, device=dev, dtype=torch.float64)
        ns = max(e0.nsup, 1)
        self.conf = torch.zeros(R, ns * ns, device=dev, dtype=torch.int32)
        self.ws = None
        self.ws_B = 0
        self._plans = {}
        self._bound_this_epoch = False  # fit(): parameter bindings checked once per fit
        for r, (e, (oA, oB)) in enumerate(zip(self.engines, self.optimizers)):
            e.attach_pack(self, r)
            e.bind_optimizer("A", oA)
            e.bind_optimizer("B", oB)
        # BatchNorm num_batches_tracked of every replica as a 0-d view of one [R] tensor, so a
        # packed launch chain advances all of them with one add instead of R small launches
        self._mod_dicts = _module_dicts(self.models)  # for fit()'s end-of-epoch module modes
        self.nbt = torch.zeros(R, device=dev, dtype=torch.long)
        for r, e in enumerate(self.engines):
            bn = e.dgcnn.BN1
            with torch.no_grad():
                self.nbt[r].copy_(bn.num_batches_tracked.reshape(()))
            bn.num_batches_tracked = self.nbt[r]

    @staticmethod
    def _shape(e):
        return (e.p, e.L, e.K, e.nsup, e.h, e.F, e.n, e.H, e.sig, e.ecc)

    def moments(self, g, r):
        return self.m[g][r], self.v[g][r]

    # ------------------------------------------------------------------ launch plumbing
    def _dims(self, Bmax, T):
        d = self.engines[0].dims(Bmax, T)
        d.R = self.R
        return d

    def check_device_status(self, where="check"):
        """Raise if a merged-backward hand-off wait of any replica timed out since the last check
        (synchronises; the packed fit checks once per epoch inside its single copy back)."""
        if self.ws is not None:
            v = nat.status_view(self.ws, self.ws_off, self.R)
            nat.raise_on_status(v.cpu().numpy(), v, where)

    def _workspace(self, Bmax, T):
        if self.ws is None or self.ws_B < Bmax:
            self.check_device_status("workspace growth")
            d = self._dims(Bmax, T)
            nbytes = nat.lib().redcliff_workspace_bytes(ctypes.byref(d))
            if nbytes == 0:
                nat.check(-1, "workspace_bytes")
            self.ws = torch.zeros(nbytes // 4, device=self.device, dtype=torch.float32)
            self.ws_B = Bmax
            self.ws_off = nat.workspace_layout(d)
        return self._dims(self.ws_B, T)

    def _hyper(self):
        if self._bound_this_epoch:
            # inside fit(): nothing changes a coefficient, learning rate or BatchNorm setting of
            # a replica, so the [R] hyper-parameter rows built at the fit's first launch stand
            # (R key computations per launch were ~1 ms of host time per epoch at R = 128)
            return self._with_offsets(self._hyper_cat)
        parts = [e._hyper() for e in self.engines]
        key = tuple(e.hyper_key for e in self.engines)
        if key != getattr(self, "_hyper_key", None):
            self._hyper_cat = torch.cat(parts).contiguous()
            self._hyper_key = key
        return self._with_offsets(self._hyper_cat)

    # byte offsets of RedcliffReplicaHyper.{A,B}.t_offset (include/redcliff_hip.h)
    _HSIZE = ctypes.sizeof(nat.ReplicaHyper)
    _TOFF = (nat.ReplicaHyper.A.offset + nat.AdamHyper.t_offset.offset,
             nat.ReplicaHyper.B.offset + nat.AdamHyper.t_offset.offset)

    def _with_offsets(self, base):
        """The hyper rows `base` with every replica's Adam step offsets (self._toff [R][2], the
        replica's step number minus its launch's) written in; the device copy is rebuilt only when
        an offset changes (a replica crosses a phase boundary of a mixed-schedule pack)."""
        toff = getattr(self, "_toff", None)
        if toff is None or not toff.any():
            return base
        key = (base.data_ptr(), toff.tobytes())
        cur = getattr(self, "_hyper_off", None)
        if cur is None or cur[0] != key:
            raw = base.cpu().numpy().reshape(self.R, self._HSIZE).copy()
            for gi in (0, 1):
                o = self._TOFF[gi]
                raw[:, o:o + 4] = np.ascontiguousarray(toff[:, gi], dtype=np.int32).view(np.uint8).reshape(self.R, 4)
            cur = (key, torch.from_numpy(raw.reshape(-1)).to(self.device))
            self._hyper_off = cur
        return cur[1]

    def _active_list(self, active):
        """(host int32 array or None, engines stepped)"""
        if active is None:
            return None, self.engines
        act = np.ascontiguousarray(sorted(int(r) for r in active), dtype=np.int32)
        return act, [self.engines[r] for r in act]

    def _args(self, d, flags, nbn, ds, stats, active=None):
        a = nat.StepArgs()
        a.d = d
        a.flags = flags | nat.REFRESH_SUPPORTS  # the pack's workspace holds its own supports
        a.n_bn_updates = nbn
        act, engs = self._active_list(active)
        # Adam step numbers: the launch carries the smallest of the active replicas' (+1) and every
        # replica's hyper row its difference from it (t_offset): replicas of a mixed-schedule pack
        # may have stepped a group different numbers of times.  Replicas that stopped early keep
        # theirs and are not in the active list.
        ts = []
        idx = list(range(self.R)) if act is None else [int(r) for r in act]
        for gi, (g, bit) in enumerate((("A", nat.STEP_A), ("B", nat.STEP_B))):
            t = [e.opt[g]["t"] if e.opt[g] is not None else 0 for e in engs]
            t0 = min(t) if t else 0
            ts.append(t0 + 1)
            if (flags & bit) and any(x != t0 for x in t):
                if getattr(self, "_toff", None) is None:
                    self._toff = np.zeros((self.R, 2), dtype=np.int64)
            if (flags & bit) and getattr(self, "_toff", None) is not None:
                self._toff[idx, gi] = np.asarray(t, dtype=np.int64) - t0
        a.tA, a.tB = ts
        # data: one dataset for the whole grid (strides 0), or per-replica data sets (PerReplica)
        a.X, a.x_rstride = ds["X"].data_ptr(), ds.get("xr", 0)
        a.labels, a.lab_rstride = (ds["lab"].data_ptr() if ds.get("lab") is not None else None), ds.get("labr", 0)
        a.bn_stats = stats.data_ptr() if stats is not None else None
        a.bn_stats_rstride = ds.get("statsr", 0) if stats is not None else 0
        a.emb, a.emb_stride = self.emb.data_ptr(), self.emb.shape[1]
        a.fac, a.fac_stride = self.fac.data_ptr(), self.fac.shape[1]
        a.emb_m, a.emb_v = self.m["A"].data_ptr(), self.v["A"].data_ptr()
        a.fac_m, a.fac_v = self.m["B"].data_ptr(), self.v["B"].data_ptr()
        a.bn_rm, a.bn_rv = self.bn[0].data_ptr(), self.bn[1].data_ptr()
        self._hyper_dev = self._hyper()
        a.hyper = self._hyper_dev.data_ptr()
        a.ws, a.ws_bytes = self.ws.data_ptr(), self.ws.numel() * 4
        a.acc = self.acc.data_ptr()
        a.confusion = self.conf.data_ptr()
        if act is not None:
            self._act_keep = act  # the host array must outlive the call
            a.replicas = act.ctypes.data_as(ctypes.c_void_p)
            a.n_replicas = len(act)
        return a, engs

    def _index(self, idx):
        """Device index tensor of replica indices, cached per index set: building it from a python
        list is a pageable host-to-device copy, which blocks the host until the stream drains."""
        key = tuple(int(i) for i in idx)
        cache = self.__dict__.setdefault("_idx_cache", {})
        t = cache.get(key)
        if t is None:
            if len(cache) > 64:
                cache.clear()
            t = cache[key] = torch.as_tensor(np.asarray(key, dtype=np.int64)).to(self.device)
        return t

    def _mask(self, active):
        """[R] long device tensor: 1 for the active replicas (all when None), cached per set."""
        key = ("mask",) + (tuple(range(self.R)) if active is None else tuple(sorted(int(i) for i in active)))
        cache = self.__dict__.setdefault("_idx_cache", {})
        t = cache.get(key)
        if t is None:
            m = np.zeros(self.R, dtype=np.int64)
            m[list(key[1:])] = 1
            t = cache[key] = torch.as_tensor(m).to(self.device)
        return t

    def _state_tensors(self):
        """(name, tensor, replica dim) of everything a training epoch advances per replica."""
        return [("emb", self.emb, 0), ("fac", self.fac, 0), ("mA", self.m["A"], 0), ("vA", self.v["A"], 0),
                ("mB", self.m["B"], 0), ("vB", self.v["B"], 0), ("bn", self.bn, 1), ("nbt", self.nbt, 0)]

    def _save_state(self, full=True):
        """The state a training epoch advances, copied aside before the next epoch runs
        speculatively.  full=False copies only what best-model snapshots read (parameters,
        BatchNorm statistics): enough when no replica can stop at this epoch, i.e. nothing will
        be rolled back (the Adam moments are 2/3 of the bytes: R = 128 D4IC, ~95 of 144 us)."""
        if getattr(self, "_prev", None) is None:
            self._prev = dict((n, torch.empty_like(t)) for n, t, _ in self._state_tensors())
        with torch.no_grad():
            for n, t, _ in self._state_tensors():
                if full or n in ("emb", "fac", "bn", "nbt"):
                    self._prev[n].copy_(t)
        self._prev_full = full

    def _step_counts(self, r):
        e = self.engines[r]
        return tuple(None if e.opt[g] is None else e.opt[g]["t"] for g in ("A", "B"))

    def _roll_back(self, reps, steps_before):
        """Replicas `reps` back to the state saved by _save_state (a speculative epoch undone)."""
        if not getattr(self, "_prev_full", False):
            raise RuntimeError("packed fit: rollback without a full saved state (stop-rule bookkeeping out of step)")
        idx = self._index(sorted(reps))
        with torch.no_grad():
            for n, t, dim in self._state_tensors():
                t.index_copy_(dim, idx, self._prev[n].index_select(dim, idx))
            # hand-off timeouts logged by the undone epoch go with its gradients
            nat.status_view(self.ws, self.ws_off, self.R).index_fill_(0, idx, 0)
        for r in reps:
            e = self.engines[r]
            for g, t in zip(("A", "B"), steps_before[r]):
                if t is not None:
                    e.opt[g]["t"] = t
            e._sync_steps()
            e.supports_fresh = False

    def _ensure_bound(self):
        if not self._bound_this_epoch:
            for e in self.engines:
                e.ensure_bound()

    def cache_dataset(self, loader):
        """Upload a training / validation set once; see FitEngine.cache_dataset.  A ``PerReplica``
        list of R loaders becomes one [R][N][T][p] window tensor (labels [R][N][K], BatchNorm batch
        statistics [R][nbatch][2][F], one launch), read through the kernels' replica strides."""
        if isinstance(loader, PerReplica):
            return self._cache_per_replica(loader)
        return self.engines[0].cache_dataset(loader)

    def _cache_per_replica(self, loaders):
        from .engine import select_labels
        key = tuple(id(x) for x in loaders)
        cache = self.__dict__.setdefault("_pr_cache", {})
        if key in cache:
            return cache[key][1]
        if len(loaders) != self.R:
            raise ValueError("PerReplica data: %d loaders for %d replicas" % (len(loaders), self.R))
        e0 = self.engines[0]
        xs_all, labs_all, sizes0 = [], [], None
        for r, loader in enumerate(loaders):
            xs, ys, sizes = [], [], []
            for X, Y in loader:
                xs.append(X.to(torch.float32))
                ys.append(select_labels(Y, e0.K, e0.Lmax) if Y is not None else torch.zeros(X.shape[0], e0.K))
                sizes.append(int(X.shape[0]))
            if sizes0 is None:
                sizes0 = sizes
            elif sizes != sizes0:
                raise ValueError("PerReplica data: replica %d's batches %s differ from replica 0's %s (a pack's "
                                 "replicas step the same batch sequence)" % (r, sizes, sizes0))
            xs_all.append(torch.cat(xs, 0))
            labs_all.append(torch.cat(ys, 0).to(torch.float32))
        shapes = set(tuple(x.shape) for x in xs_all)
        if len(shapes) != 1:
            raise ValueError("PerReplica data: window shapes differ across replicas: %s" % sorted(shapes))
        X = torch.stack(xs_all).to(self.device).contiguous()  # [R][N][T][p]
        lab = torch.stack(labs_all).to(self.device).contiguous()  # [R][N][K]
        R, N, T, p = X.shape
        if p != e0.p:
            raise ValueError("expected %d channels, got %d" % (e0.p, p))
        rows = np.cumsum([0] + sizes0[:-1]).astype(np.int64)
        nb = len(sizes0)
        stats = torch.empty(R, nb, 2, e0.F, device=self.device, dtype=torch.float64)
        d = self._dims(max(sizes0), T)
        if all(s == sizes0[0] for s in sizes0[:-1]) and sizes0[-1] <= sizes0[0]:
            nat.check(nat.lib().redcliff_bn_batch_stats(ctypes.byref(d), ctypes.c_void_p(X.data_ptr()), N * T * p, N,
                                                        sizes0[0], ctypes.c_void_p(stats.data_ptr()), nb * 2 * e0.F,
                                                        _stream()), "bn_batch_stats (per replica)")
        else:
            for i, (r0, s) in enumerate(zip(rows, sizes0)):
                nat.check(nat.lib().redcliff_bn_batch_stats(
                    ctypes.byref(d), ctypes.c_void_p(X[0, r0].data_ptr()), N * T * p, s, s,
                    ctypes.c_void_p(stats[0, i].data_ptr()), nb * 2 * e0.F, _stream()), "bn_batch_stats (per replica)")
        ds = {"X": X, "lab": lab, "rows": rows, "sizes": np.asarray(sizes0, dtype=np.int32), "stats": stats,
              "T": int(T), "Bmax": max(sizes0), "len": nb, "loader": loaders, "per_replica": True,
              "xr": N * T * p, "labr": N * e0.K, "statsr": nb * 2 * e0.F}
        cache[key] = (loaders, ds)  # the loaders stay referenced, so their ids stay unique
        return ds

    @staticmethod
    def _stats_at(ds, b0, nb=None):
        """The BatchNorm batch statistics of ds from batch b0 on ([R][..] per replica, shared
        otherwise): the kernels advance 2F doubles per step and a replica stride of ds["statsr"]."""
        st = ds["stats"]
        if ds.get("per_replica"):
            return st[:, b0:] if nb is None else st[:, b0:b0 + nb]
        return st[b0:] if nb is None else st[b0:b0 + nb]

    # ------------------------------------------------------------------ stepping
    def run_steps(self, kinds, ds, rows=None, sizes=None, stats=None, active=None):
        """Update kinds of one phase over consecutive batches of `ds` for the active replicas
        (all when None): one redcliff_train_steps launch chain of R-replica kernels per kind."""
        self._ensure_bound()
        rows = ds["rows"] if rows is None else rows
        sizes = ds["sizes"] if sizes is None else sizes
        stats = ds["stats"] if stats is None else stats  # a view starting at the first step's batch
        d = self._workspace(max(int(ds["Bmax"]), 1), ds["T"])
        for kind in kinds:
            flags, nbn = flags_for(kind, self.engines[0].nsup)
            a, engs = self._args(d, flags, nbn, ds, stats if flags & nat.BN_TRAIN else None, active)
            rows_a = np.ascontiguousarray(rows, dtype=np.int64)
            sizes_a = np.ascontiguousarray(sizes, dtype=np.int32)
            nat.check(nat.lib().redcliff_train_steps(ctypes.byref(a), len(rows_a),
                                                     rows_a.ctypes.data_as(ctypes.c_void_p),
                                                     sizes_a.ctypes.data_as(ctypes.c_void_p), 2 * self.engines[0].F,
                                                     _stream()), "packed train_steps")
            for e in engs:
                e._after(flags, nbn, len(rows_a), bn=False)
            if nbn:
                with torch.no_grad():
                    self.nbt.add_(self._mask(active), alpha=nbn * len(rows_a))
            for e in self.engines:
                e.supports_fresh = False  # the single-fit workspace's supports are stale now

    def phase_groups(self, epoch, active=None):
        """{update kinds: [replicas]} of `epoch` (...withStateSmoothing.py:741-759) for the active
        replicas, in the order of each group's first replica."""
        idx = range(self.R) if active is None else sorted(int(r) for r in active)
        groups = {}
        for r in idx:
            groups.setdefault(tuple(phase_of_epoch(self.models[r], epoch)), []).append(r)
        return groups

    def run_epoch(self, epoch, ds, active=None, set_modes=True):
        """The batch_update phase of `epoch` (...withStateSmoothing.py:741-759) over every batch
        of `ds`, for the active replicas.  Replicas whose schedules put them in different phases
        this epoch run as one launch chain per phase group (the replicas are independent, so the
        order of the groups changes no result).  Returns {kinds: replicas}."""
        groups = self.phase_groups(epoch, active)
        for kinds, reps in groups.items():
            act = active if len(groups) == 1 else reps
            if len(kinds) <= 1:
                self.run_steps(list(kinds), ds, active=act)
            else:  # several updates per batch: batch-major order as in batch_update
                for bi, (r, s) in enumerate(zip(ds["rows"], ds["sizes"])):
                    for kind in kinds:
                        self.run_steps([kind], ds, [r], [s], self._stats_at(ds, bi, 1), active=act)
            if set_modes:
                for r in reps:
                    self.models[r]._set_module_modes(kinds[-1] if kinds else None)
        return groups

    def _values(self, ds, active=None, host=True):
        """validate_training accumulators of the active replicas: raw acc [R][8], confusion
        (host=False: the device buffers, for one combined copy back)."""
        self._ensure_bound()
        self.acc.zero_()
        self.conf.zero_()
        e0 = self.engines[0]
        d = self._workspace(max(int(ds["Bmax"]), 1), ds["T"])
        flags = nat.VALUES | (nat.CONFUSION if e0.nsup > 0 else 0)
        a, _ = self._args(d, flags, 0, ds, None, active)
        rows_a = np.ascontiguousarray(ds["rows"], dtype=np.int64)
        sizes_a = np.ascontiguousarray(ds["sizes"], dtype=np.int32)
        nat.check(nat.lib().redcliff_train_steps(ctypes.byref(a), len(rows_a), rows_a.ctypes.data_as(ctypes.c_void_p),
                                                 sizes_a.ctypes.data_as(ctypes.c_void_p), 2 * e0.F, _stream()),
                  "packed validate")
        ns = max(e0.nsup, 1)
        if not host:
            return self.acc, self.conf
        return self.acc.cpu().numpy(), self.conf.cpu().numpy().reshape(self.R, ns, ns)

    def validate(self, ds, active=None):
        """validate_training loss averages (:1650-1790) of every replica: array [R][7]
        (forecast, factor, cos, fw_l1, smooth, adj, combo), plus confusion matrices [R][nsup][nsup]."""
        acc, conf = self._values(ds, active)
        nb = np.maximum(acc[:, 7:8], 1.0)
        return acc[:, :7] / nb, conf

    def embed_raw(self, X, active=None):
        """Raw embedder outputs [Ra][B][K] of windows X (B, T >= Lmax, p) -- or per replica,
        X (R, B, T, p) -- for the active replicas (BatchNorm running statistics): one
        embedder-only launch for all of them."""
        X = X.to(self.device, torch.float32).contiguous()
        B, T, p = X.shape[-3:]
        d = self._workspace(max(B, 1), T)
        ds = {"X": X, "lab": None, "xr": B * T * p if X.dim() == 4 else 0}
        a, _ = self._args(d, 0, 0, ds, None, active)
        a.B, a.row0 = B, 0
        nat.check(nat.lib().redcliff_train_step(ctypes.byref(a), _stream()), "packed embed")
        idx = list(range(self.R)) if active is None else sorted(active)
        K = self.engines[0].K
        o, tot = self.ws_off["w"], self.ws_off["total"]
        ws = self.ws[:self.R * tot].view(self.R, tot)
        return ws[:, o:o + B * K].index_select(0, self._index(idx)).view(len(idx), B, K)

    def gc_norms(self):
        """(G [R][K][p][p][L], G0 [R][K][p][p]) of every replica's factor weights (one launch)."""
        e0 = self.engines[0]
        d = nat.Dims(R=self.R, Bmax=1, T=e0.L, p=e0.p, L=e0.L, K=e0.K, h=e0.h, F=e0.L, n=1, H=1, M1=1, nsup=0,
                     use_sigmoid=0, sigmoid_ecc=0.0)
        G = torch.empty(self.R, e0.K, e0.p, e0.p, e0.L, device=self.device, dtype=torch.float32)
        G0 = torch.empty(self.R, e0.K, e0.p, e0.p, device=self.device, dtype=torch.float32)
        nat.check(nat.lib().redcliff_gc_norms(ctypes.byref(d), ctypes.c_void_p(self.fac.data_ptr()),
                                              self.fac.shape[1], ctypes.c_void_p(G.data_ptr()),
                                              ctypes.c_void_p(G0.data_ptr()), _stream()), "packed gc_norms")
        return G, G0

    # ------------------------------------------------------------------ packed fit
    def fit(self, *args, **kwargs):
        """R fits of ``fit()`` in one packed launch chain; see ``_fit``.  The host side of an epoch
        is O(R) python, so the cyclic garbage collector is paused for the fit: its full passes
        over R models' module trees cost as much as whole epochs (restored afterwards)."""
        return fit_packs([(self, args, kwargs)])[0]

    def _fit(self, *args, **kwargs):
        """The packed fit run to completion (no interleaving with other packs)."""
        g = self._fit_steps(*args, **kwargs)
        while True:
            try:
                next(g)
            except StopIteration as e:
                return e.value

    def _fit_steps(self, save_dir, X_train, X_val, max_iter, lookback=5, check_every=50, verbose=0, GC=None,
             deltaConEps=0.1, in_degree_coeff=1., out_degree_coeff=1., stopping_criteria_forecast_coeff=1.,
             stopping_criteria_factor_coeff=1., stopping_criteria_cosSim_coeff=1., output_length=1, save_plots=False,
             cost_criteria="CosineSimilarity", unsupervised_start_index=0, max_factor_prior_batches=10):
        """R fits of ``fit()`` (...withStateSmoothing.py:1175-1647) in one packed launch chain, as a
        generator: it yields whenever its device work for the next host decision is enqueued and the
        host would otherwise wait for it (once per epoch, and before the final copy back), so
        ``fit_packs`` can interleave several packs -- each on its own stream -- and the GPU runs
        their epochs concurrently.  The return value (StopIteration.value) is the fit's.

        Every replica follows exactly the rules (and the host code, FitTracker) of a single fit:
        its histories, its stopping criterion (per-model stopping_criteria_* may be given as
        lists), its own phase schedule (num_pretrain_epochs / num_acclimation_epochs /
        training_mode of its model), best-epoch snapshot, checkpoints every check_every epochs
        (save_dir: a list of R directories, or one root that gets replica_<r>/ sub-directories),
        restore_parameters and final model file.  X_train / X_val / GC may be ``PerReplica``
        (each replica fits its own data set against its own true graphs).  A stopped replica
        leaves the active list: nothing of it is launched or updated afterwards.  Returns the
        final validation combo loss of every replica; each model gets ``fit_history`` as a single
        fit would."""
        if output_length != 1:
            raise NotImplementedError("output_length must be 1")
        t_in = time.perf_counter()
        R, models = self.R, self.models
        for m in models:
            if not m.fused_supported() or "Freeze" in m.training_mode or m.__dict__.get("_factors_detached"):
                raise NotImplementedError("packed fits cover the fused (published) configuration")
        modes = set(m.primary_gc_est_mode for m in models)
        if len(modes) != 1:
            raise ValueError("a packed fit tracks GC progress in one primary_gc_est_mode, got %s" % sorted(modes))

        def per(x):
            return list(x) if isinstance(x, (list, tuple)) else [x] * R
        if isinstance(GC, PerReplica) and len(GC) != R:
            raise ValueError("PerReplica GC: %d graph lists for %d replicas" % (len(GC), R))
        gc_of = (lambda r: GC[r]) if isinstance(GC, PerReplica) else (lambda r: GC)
        scf, scfa, scc = per(stopping_criteria_forecast_coeff), per(stopping_criteria_factor_coeff), \
            per(stopping_criteria_cosSim_coeff)
        dirs = None
        if save_dir is not None:
            dirs = list(save_dir) if isinstance(save_dir, (list, tuple)) else \
                [os.path.join(save_dir, "replica_%d" % r) for r in range(R)]
        trackers = [FitTracker(m, gc_of(r), deltaConEps, in_degree_coeff, out_degree_coeff, scf[r], scfa[r], scc[r],
                               lookback, check_every) for r, m in enumerate(models)]
        e0, m0 = self.engines[0], models[0]
        nsup, p, K = e0.nsup, e0.p, e0.K
        Lm, ls = m0.Lmax, min(m0.gen_lag, m0.embed_lag)
        train = self.cache_dataset(X_train)
        val = self.cache_dataset(X_val)
        self._workspace(max(int(train["Bmax"]), int(val["Bmax"]), 1), train["T"])
        dev_metrics = (m0.wavelet_level is None and 2 <= p <= 64
                       and m0.primary_gc_est_mode in ("conditional_factor_exclusive", "conditional_factor_fixed_embedder"))
        if not dev_metrics:
            raise NotImplementedError("packed fits track GC progress on the device (no wavelet_level, 2 <= p <= 64, "
                                      "conditional modes); fit these models one by one")
        best = _PackBest(self)
        hlog = DeferredHistories()
        active = list(range(R))
        nfirst = min(int(val["sizes"][0]), m0.MAX_NUM_SAMPS_FOR_GC_PROGRESS_TRACKING)
        # GC tracking windows: the first validation batch's first samples (:1366-1370), per replica
        # when every replica has its own validation set
        Xv = val["X"][:, :nfirst, :Lm, :].contiguous() if val.get("per_replica") else val["X"][:nfirst, :Lm, :]
        gc_lists = {}  # PerReplica GC: the active replicas' true-graph lists, one list object per active set

        def truths(act):
            k = tuple(act)
            if k not in gc_lists:
                gc_lists.clear()
                gc_lists[k] = [GC[r] for r in act]
            return gc_lists[k]
        # The module train/eval flags -- which no fused launch reads -- are set once, to the state
        # the reference leaves after every epoch (eval: GC tracking and validation call .eval()),
        # before checkpoints and at the end, instead of walking R module trees twice per epoch.
        # nothing inside the loop re-points a parameter (snapshots and checkpoints copy), so the
        # bindings of all R engines are checked once per fit, not per launch
        self._bound_this_epoch = False
        self._ensure_bound()
        self._hyper_key = None
        self._hyper()  # the fit's hyper-parameter rows (fixed from here on, see _hyper)
        self._bound_this_epoch = True
        # Overlap: while the host digests epoch `it` (trackers, stopping rule, snapshots), the GPU
        # already trains epoch it + 1 for the replicas still active (speculatively).  The state
        # every training epoch advances is copied aside first (`_save_state`); best-model
        # snapshots of epoch `it` are taken from that copy, and a replica that stops at `it` is
        # rolled back to it (parameters, Adam moments and step counts, BatchNorm statistics), so
        # every replica ends exactly where its own fit() would.  No speculation across a
        # checkpoint epoch (the files hold epoch `it`'s state) or past max_iter.
        # "pretrain_factor" modes re-order each fit's factors before epoch num_pretrain_epochs
        # (...withStateSmoothing.py:1318-1326, initialize_factors_with_prior with fit()'s cost_criteria,
        # unsupervised_start_index and max_factor_prior_batches)
        reorder_at = dict((r, m.num_pretrain_epochs) for r, m in enumerate(models) if "pretrain_factor" in m.training_mode)
        reorder_epochs = set(reorder_at.values())

        def launch_train(ep):
            if ep in reorder_epochs:
                for r in active:  # with the caller's settings, as each single fit's _prior_hook passes them
                    if reorder_at.get(r) != ep:
                        continue
                    xr = X_train[r] if isinstance(X_train, PerReplica) else X_train
                    models[r].initialize_factors_with_prior(X_train=xr, cost_criteria=cost_criteria,
                                                            unsupervised_start_index=unsupervised_start_index,
                                                            max_batches=max_factor_prior_batches)
            self.conf.zero_()
            self.run_epoch(ep, train, active, set_modes=False)

        # REDCLIFF_PACK_PROFILE=1: host seconds per epoch in (enqueue of the evaluation, enqueue of
        # the next epoch's training, waiting for the device, digesting the epoch) -> self.last_profile
        prof = [] if os.environ.get("REDCLIFF_PACK_PROFILE", "0") != "0" else None
        self.last_profile = prof
        t_loop = time.perf_counter()
        try:
            it = 0
            if max_iter > 0:
                launch_train(0)
            while it < max_iter and active:
                if prof is not None:
                    tp = [time.perf_counter()]
                if verbose:
                    print("ReplicaPack.fit: epoch %d, %d of %d replicas active" % (it, len(active), R), flush=True)
                tr_act = [trackers[r] for r in active]
                # ---- the per-epoch evaluation of every active replica on the device, ONE copy
                # back: train confusion, GC progress on the first validation batch (:1366-1414),
                # validation (:1416-1480, one launch chain)
                with torch.no_grad():
                    conf_d = self.conf.clone()
                    w_raw = self.embed_raw(Xv, active)  # (Ra, S, K)
                    emb0 = models[0].factor_score_embedder
                    w = torch.sigmoid(emb0.sigmoid_eccentricity_coeff * w_raw) if emb0.use_sigmoid_restriction else w_raw
                    G, G0 = self.gc_norms()
                    A = self.emb[:, :p * p].view(R, p, p)
                    if len(active) < R:  # the active replicas' rows (all of them: no gather needed)
                        ai = self._index(active)
                        G, G0, A = G[ai], G0[ai], A[ai]
                    est_t, nolag_t = conditional_gc_estimates(w, G, G0, A, nsup, ls, m0.primary_gc_est_mode)
                    Ra, S = est_t.shape[0], est_t.shape[1]
                    vals_d = None
                    if GC is not None and nsup > 0 and S > 0:
                        est_flat = est_t.reshape(Ra * S, *est_t.shape[2:])
                        if isinstance(GC, PerReplica):  # each replica scored against its own true graphs
                            vals_d = M.gc_progress_values_grouped(truths(active), est_flat, S, deltaConEps,
                                                                  in_degree_coeff, out_degree_coeff, host=False)
                        else:
                            vals_d = M.gc_progress_values(GC, est_flat, deltaConEps, in_degree_coeff,
                                                          out_degree_coeff, host=False)
                    l1_d, dots_d = M.gc_track_values(est_t, nolag_t, host=False)
                    acc_d, confv_d = self._values(val, active, host=False)
                    pending = M.fetch_async([conf_d, l1_d, dots_d, acc_d, confv_d,
                                             nat.status_view(self.ws, self.ws_off, R)] +
                                            ([vals_d] if vals_d is not None else []))
                if prof is not None:
                    tp.append(time.perf_counter())
                spec = (it + 1 < max_iter and not (dirs is not None and it % check_every == 0)
                        and it + 1 not in reorder_epochs)
                if spec:
                    # a replica can stop at this epoch only after pretraining / acclimation and when
                    # its last improvement is exactly lookback * check_every epochs back (FitTracker.step)
                    can_stop = any(trackers[r].may_stop(it) for r in active)
                    self._save_state(full=can_stop)
                    steps_before = [self._step_counts(r) for r in range(R)]
                    launch_train(it + 1)
                if prof is not None:
                    tp.append(time.perf_counter())
                yield  # the epoch's work is enqueued: let other packs enqueue theirs before waiting
                got = pending.wait()
                if prof is not None:
                    tp.append(time.perf_counter())
                cms, l1, dots, acc, conf = got[:5]
                nat.raise_on_status(got[5], nat.status_view(self.ws, self.ws_off, R), "packed fit epoch %d" % it)
                vals = got[6].reshape(Ra, S, *got[6].shape[1:]) if vals_d is not None else None
                if nsup > 0:
                    train_confusion_many(tr_act, cms.reshape(R, nsup, nsup)[active], log=hlog, cols=active)
                gc_progress_many(tr_act, vals, *M.track_values_finish(l1, dots), log=hlog, cols=active)
                ns = max(nsup, 1)
                conf = conf.reshape(R, ns, ns)
                nb = float(val["len"])
                rates = confusion_rates_many(conf[active]) if nsup > 0 else None
                for i, r in enumerate(active):
                    hist = [[] for _ in range(5)] if nsup > 0 else [None] * 5
                    rt = tuple(x[i].copy() for x in rates) if nsup > 0 else None
                    trackers[r].validation(models[r]._validation_tuple(acc[r], nb, conf[r], *hist, rates=rt))
                # ---- early stopping, per replica (:1482-1559); snapshots copied in one batch
                stopped = []
                for r in active:
                    if trackers[r].step(it, lambda r=r: best.mark(r)):
                        stopped.append(r)
                best.copy_marked(self._prev if spec else None)
                for r in stopped:
                    if verbose:
                        print("ReplicaPack.fit: replica %d stops early at epoch %d" % (r, it), flush=True)
                if spec and stopped:
                    self._roll_back(stopped, steps_before)
                active = [r for r in active if r not in stopped]
                if dirs is not None and it % check_every == 0:
                    hlog.flush()
                    _eval_modes(models, self._mod_dicts)
                    for r in active:
                        trackers[r].checkpoint(dirs[r], it, optimizers=self.optimizers[r], save_plots=save_plots)
                it += 1
                if not spec and it < max_iter and active:
                    launch_train(it)
                if prof is not None:
                    tp.append(time.perf_counter())
                    prof.append([b - a for a, b in zip(tp, tp[1:])])
            t_end_loop = time.perf_counter()
            # ---- restore best parameters and the final validation (:1621-1647), enqueued first
            # (the bindings checked at the fit's start still hold); the host flushes the deferred
            # histories and writes the module modes while they run
            snaps = [t.best_model for t in trackers]
            if all(isinstance(b, _PackSnapshot) and b._best is best and b._r == r for r, b in enumerate(snaps)):
                with torch.no_grad():  # every replica's restore_parameters as two row-wise copies
                    self.emb.copy_(best.emb)
                    self.fac.copy_(best.fac)
            else:
                for r, m in enumerate(models):
                    restore_parameters(m, snaps[r])
            for e in self.engines:
                e.supports_fresh = False
            final = M.fetch_async(list(self._values(val, host=False)))
        finally:
            self._bound_this_epoch = False
        hlog.flush()
        _eval_modes(models, self._mod_dicts)
        yield
        acc, conf = final.wait()
        conf = conf.astype(np.int32).reshape(R, max(nsup, 1), max(nsup, 1))
        for r, m in enumerate(models):
            if dirs is not None:
                os.makedirs(dirs[r], exist_ok=True)
                torch.save(standalone_copy(m), os.path.join(dirs[r], "final_best_model.bin"))
        nb = float(val["len"])
        finals = []
        for r, m in enumerate(models):
            hist = [[] for _ in range(5)] if nsup > 0 else [None] * 5
            v = m._validation_tuple(acc[r], nb, conf[r], *hist)
            finals.append(v[-6] if nsup > 0 else v[-1])
            m.fit_history = trackers[r].history()
        if prof is not None:  # host seconds before the epoch loop, in it, after it
            self.last_profile_edges = (t_loop - t_in, t_end_loop - t_loop, time.perf_counter() - t_end_loop)
        return finals


def fit_packs(jobs):
    """Several packed fits at once: jobs = [(pack, args, kwargs)] of ``ReplicaPack.fit``.  Each pack
    runs on its own stream; every pack's epoch is enqueued before any host waits for a result
    (ReplicaPack._fit_steps yields there), so the device runs the packs' epochs concurrently.  This
    is for a GPU's share of a grid whose shape classes are small packs -- the synthetic grid's (K, p)
    classes hold 15 to 105 data sets (train/REDCLIFF_S_CMLP_synSysInnovGauss1030_BSCgsSmooth3Parsim.py:
    140-1131) -- where one small pack's latency-bound epoch leaves most of the chip idle.  Every pack's
    arithmetic is unchanged (the same launches, on another stream), so each replica ends exactly as
    in its pack's own fit.  Returns the packs' fit results in job order.

    Concurrency is per pack stream, with one limit: a pack of 32 or more replicas forks its factor
    chain onto the library's auxiliary stream, and there is ONE of those per host thread and device
    (rc_capi.hip g_aux, with its fork / join events), so the forked factor chains of several large
    packs run one after another on it while their embedder chains overlap on the packs' own
    streams.  A share of the reference grids holds at most two packs that large (the TST grid's
    256-point classes, shard_grid); the synthetic grid's classes stay below the fork threshold."""
    gc_was = gc.isenabled()
    gc.disable()
    cur = torch.cuda.current_stream()
    try:
        if len(jobs) == 1:
            pack, args, kwargs = jobs[0]
            return [pack._fit(*args, **kwargs)]
        run = []
        for i, (pack, args, kwargs) in enumerate(jobs):
            s = torch.cuda.Stream(device=pack.device)
            s.wait_stream(cur)  # the packs' state was written on the caller's stream
            with torch.cuda.stream(s):
                run.append([i, pack, s, pack._fit_steps(*args, **kwargs)])
        out = [None] * len(jobs)
        while run:
            for job in list(run):
                i, pack, s, g = job
                with torch.cuda.stream(s):
                    try:
                        next(g)
                    except StopIteration as e:
                        out[i] = e.value
                        run.remove(job)
                        cur.wait_stream(s)  # the caller's stream sees the pack's final state
        return out
    finally:
        if gc_was:
            gc.enable()


def _module_dicts(models):
    """The __dict__ of every submodule of the embedders and factors of `models` (the modules
    whose train flags fit() leaves False), walked once with an explicit stack."""
    out, stack = [], []
    for m in models:
        stack.append(m.factor_score_embedder)
        stack.extend(m.factors)
    while stack:
        d = stack.pop().__dict__
        out.append(d)
        stack.extend(c for c in d["_modules"].values() if c is not None)
    return out


def _eval_modes(models, dicts=None):
    """The module modes every fit epoch ends in (GC tracking + validate_training call .eval() on
    the embedder and every factor, ...withStateSmoothing.py:1366-1480).  The flags are written
    directly (Module.train(False) sets exactly this attribute on every submodule; no module of
    this package overrides train()): torch's recursive .eval() with its __setattr__ per module
    cost ~110 ms per 128-fit pack (28,800 modules), a fifth of a packed D4IC fit's wall clock.
    dicts: the modules' __dict__s listed when the pack was built (ReplicaPack._mod_dicts, the
    pack's fixed module trees), so the fit writes 28,800 flags without walking the trees."""
    for d in (_module_dicts(models) if dicts is None else dicts):
        if d["training"]:
            d["training"] = False


class _PackBest:
    """Best-epoch snapshots of every replica of a pack: rows of [R][...] buffers, refreshed for
    all improving replicas of an epoch with one indexed copy per buffer (instead of R model
    deep-copies).  mark(r) returns the replica's ParamSnapshot (views of its rows)."""

    def __init__(self, pack):
        self.pack = pack
        self.emb = torch.empty_like(pack.emb)
        self.fac = torch.empty_like(pack.fac)
        self.bn = torch.empty_like(pack.bn)
        dev = pack.device
        self.nbt = torch.zeros(pack.R, dtype=torch.long, device=dev)
        self.marked = []

    def mark(self, r):
        self.marked.append(r)
        return _PackSnapshot(self, r)

    def copy_marked(self, src=None):
        """src: a dict of [R][...] buffers holding the epoch's state (ReplicaPack._prev while the
        next epoch already runs), else the live pack buffers."""
        if not self.marked:
            return
        keys = sorted(set(self.marked))
        idx = self.pack._index(keys)
        pk = self.pack
        s = src if src is not None else {"emb": pk.emb, "fac": pk.fac, "bn": pk.bn, "nbt": pk.nbt}
        with torch.no_grad():
            self.emb.index_copy_(0, idx, s["emb"].index_select(0, idx))
            self.fac.index_copy_(0, idx, s["fac"].index_select(0, idx))
            self.bn.index_copy_(1, idx, s["bn"].index_select(1, idx))
            self.nbt.index_copy_(0, idx, s["nbt"].index_select(0, idx))
        self.marked = []


class _PackSnapshot(ParamSnapshot):
    """ParamSnapshot of replica r whose buffers are r's rows of a _PackBest, taken as views when
    first read (an improving replica's snapshot per epoch is then one small object)."""

    def __init__(self, best, r):  # noqa: super().__init__ is not called: the rows stand for its copies
        self.model = best.pack.models[r]
        self._best, self._r = best, r

    @property
    def emb(self):
        return self._best.emb[self._r]

    @property
    def fac(self):
        return self._best.fac[self._r]

    @property
    def bn(self):
        b, r = self._best, self._r
        return (b.bn[0][r], b.bn[1][r], b.nbt[r])


def model_shape(m):
    """The shape key of a model (ReplicaPack._shape of its engine), read from the module tree
    (no device work): p, gen_lag, K, nsup, h, DGCNN F / layers / hidden, sigmoid restriction."""
    g = m.factor_score_embedder.dgcnn.dgcnn
    emb = m.factor_score_embedder
    return (m.num_series, m.gen_lag, m.num_factors_nK, m.num_supervised_factors, m.gen_hidden[0], g.in_channels,
            g.num_layers, g.hid_channels, bool(emb.use_sigmoid_restriction),
            float(emb.sigmoid_eccentricity_coeff or 0.0))


def grid_packs(models_and_opts, max_replicas=256, key=None):
    """Group grid points (model, (optimizerA, optimizerB)) into packs of identical shapes (the
    reference's TST grid varies embed_lag and the graph-conv layers -- 6 shape classes --, and the
    pretrain / acclimation epochs, which a pack may mix,
    train/REDCLIFF_S_CMLP_tst100hzRerun1024AvgReg_gsSmooth1.py:278-309), in the grid's own order,
    at most max_replicas (<= 256, the longest active list of one launch) per pack.  key(i): an
    extra grouping key of point i -- e.g. the (N, T) shape of its data set, which the replicas of
    a pack with PerReplica data must share.  Returns [(models, optimizers, point indices)]."""
    if not 1 <= max_replicas <= 256:
        raise ValueError("max_replicas must be in 1..256")
    groups = {}
    order = []
    for i, (m, o) in enumerate(models_and_opts):
        k = model_shape(m) + (m.primary_gc_est_mode,) + ((key(i),) if key is not None else ())
        if k not in groups:
            groups[k] = []
            order.append(k)
        groups[k].append((i, m, o))
    out = []
    for k in order:
        g = groups[k]
        n = -(-len(g) // max_replicas)  # packs of this class, sized evenly
        for j in range(n):
            chunk = g[j * len(g) // n:(j + 1) * len(g) // n]
            out.append(([m for _, m, _ in chunk], [o for _, _, o in chunk], [i for i, _, _ in chunk]))
    return out


def _minmax_runs(w, cls, world, piece_cost):
    """Cut the class-ordered points (costs w, class keys cls) into at most `world` contiguous runs
    minimising the largest run cost, where a run costs the sum of its points' costs plus piece_cost
    for every class it touches (each is a pack of its own, with a pack's fixed per-epoch latency).
    Greedy filling is optimal for a given bound (a point only ever adds to the run it joins), so a
    bisection on the bound finds the optimum to within a 1e-6 relative step.  Returns the run index
    of every (ordered) point."""
    n = len(w)

    def fill(bound):
        owner = np.zeros(n, np.int64)
        g, load, last = 0, 0.0, None
        for j in range(n):
            add = w[j] + (piece_cost if cls[j] != last else 0.0)
            if load > 0.0 and load + add > bound:
                g += 1
                if g >= world:
                    return None
                load, last = 0.0, None
                add = w[j] + piece_cost
            load += add
            last = cls[j]
            owner[j] = g
        return owner

    lo = max(float(np.max(w)) + piece_cost, 0.0) if n else 0.0
    hi = float(np.sum(w)) + piece_cost * len(set(cls)) + 1.0
    best = fill(hi)
    while hi - lo > 1e-6 * hi:
        mid = 0.5 * (lo + hi)
        o = fill(mid)
        if o is None:
            lo = mid
        else:
            hi, best = mid, o
    return best


def shard_grid(n_points, world, rank, classes=None, cost=None, min_piece=0, piece_cost=None):
    """Grid-point indices of rank `rank` of `world` GPUs.

    classes=None: round-robin over the grid order, as SLURM array tasks map onto nodes
    (train/...gsSmooth1.py:157-160: task i -> parameters_to_be_parallelized[i-1]).

    classes (one hashable shape-class key per point, e.g. (K, p) of the synthetic grid or
    (embed_lag, graph-conv layers) of the TST grid): the points ordered by class (classes in order
    of first appearance, grid order within a class) and cut into `world` contiguous runs of equal
    total cost (cost[i], default 1 per point), so every GPU holds whole classes or long runs of one
    -- few, large packs per GPU instead of ~world-fold thinner packs of every class.

    min_piece: a GPU's piece of a class smaller than min(min_piece, half the class) joins the class's
    largest piece on another GPU (a handful of points would be a pack of its own, whose per-epoch
    launch chains cost about as much as a full one), at the price of a less even cost split.

    piece_cost (round 6): instead of the equal-cost cut, the contiguous runs minimise the largest run
    cost counting `piece_cost` for every class a run touches -- the fixed per-pack time of a share
    (bench.py REF_GRID_COST: a share's time is close to 0.073 s per pack + 0.65 ms per fit + 1.2 ms per
    algorithmic MFLOP of a window, fitted over all 16 shares of both reference grids); min_piece is then
    not used.  Measured against the equal-cost cut it was not better overall (bench.py REF_GRID_COST),
    so it is an option, not the default."""
    if classes is None:
        return list(range(rank, n_points, world))
    if len(classes) != n_points:
        raise ValueError("one class key per grid point")
    first = {}
    for i, c in enumerate(classes):
        first.setdefault(c, len(first))
    order = sorted(range(n_points), key=lambda i: (first[classes[i]], i))
    w = np.ones(n_points) if cost is None else np.asarray(cost, dtype=np.float64)
    if piece_cost is not None:
        owner = _minmax_runs(w[order], [classes[i] for i in order], world, float(piece_cost))
        return sorted(int(order[j]) for j in range(n_points) if owner[j] == rank)
    cum = np.cumsum(w[order])
    total = cum[-1] if n_points else 0.0
    # run g holds the points whose cumulative cost midpoint falls in [g, g+1) * total / world
    mid = cum - 0.5 * w[order]
    owner = np.minimum((mid * world / max(total, 1e-300)).astype(np.int64), world - 1)
    if min_piece > 0:
        pos = {}
        for j in range(n_points):
            pos.setdefault(classes[order[j]], []).append(j)
        for js in pos.values():
            counts = np.bincount(owner[js], minlength=world)
            big = int(np.argmax(counts))
            small = [g for g in range(world) if 0 < counts[g] < min(min_piece, len(js) / 2.0) and g != big]
            for j in js:
                if owner[j] in small:
                    owner[j] = big
    return sorted(int(order[j]) for j in range(n_points) if owner[j] == rank)
