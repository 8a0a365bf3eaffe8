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
momentum.  They share the training windows (one dataset for the whole grid, as in the
reference) and the update schedule of the step (phase flags, Adam step counters).

Each model stays a normal drop-in module: its parameters and its optimizers' state are
views of its pack row, so ``state_dict()``, ``GC()``, ``forward()`` and the single-fit
methods keep working on it between packed epochs.
"""
import ctypes

import numpy as np
import torch

from . import _native as nat
from .engine import _stream, flags_for, phase_of_epoch


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
        for r, (e, (oA, oB)) in enumerate(zip(self.engines, self.optimizers)):
            e.attach_pack(self, r)
            e.bind_optimizer("A", oA)
            e.bind_optimizer("B", oB)

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

    def _workspace(self, Bmax, T):
        if self.ws is None or self.ws_B < Bmax:
            d = self._dims(Bmax, T)
            nbytes = nat.lib().redcliff_workspace_bytes(ctypes.byref(d))
            if nbytes == 0:
                nat.check(-1, "workspace_bytes")
            self.ws = torch.zeros(nbytes // 4, device=self.device, dtype=torch.float32)
            self.ws_B = Bmax
        return self._dims(self.ws_B, T)

    def _hyper(self):
        return torch.cat([e._hyper() for e in self.engines]).contiguous()

    def _args(self, d, flags, nbn, ds, stats):
        e0 = self.engines[0]
        a = nat.StepArgs()
        a.d = d
        a.flags = flags | nat.REFRESH_SUPPORTS  # the pack's workspace holds its own supports
        a.n_bn_updates = nbn
        tA = set(e.opt["A"]["t"] for e in self.engines)
        tB = set(e.opt["B"]["t"] for e in self.engines)
        if len(tA) != 1 or len(tB) != 1:
            raise RuntimeError("packed replicas must share their Adam step counters (same update schedule)")
        a.tA, a.tB = tA.pop() + 1, tB.pop() + 1
        a.X, a.x_rstride = ds["X"].data_ptr(), 0  # one dataset for the whole grid
        a.labels, a.lab_rstride = ds["lab"].data_ptr(), 0
        a.bn_stats = stats.data_ptr() if stats is not None else None
        a.bn_stats_rstride = 0
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
        del e0
        return a

    def cache_dataset(self, loader):
        """Upload the (shared) training set once; see FitEngine.cache_dataset."""
        return self.engines[0].cache_dataset(loader)

    # ------------------------------------------------------------------ stepping
    def run_steps(self, kinds, ds, rows=None, sizes=None, stats=None):
        """Update kinds of one phase over consecutive batches of `ds` for all R replicas
        (one redcliff_train_steps launch chain of R-replica kernels per kind)."""
        for e in self.engines:
            e.ensure_bound()
        rows = ds["rows"] if rows is None else rows
        sizes = ds["sizes"] if sizes is None else sizes
        stats = ds["stats"] if stats is None else stats
        d = self._workspace(max(int(ds["Bmax"]), 1), ds["T"])
        for kind in kinds:
            flags, nbn = flags_for(kind, self.engines[0].nsup)
            a = self._args(d, flags, nbn, ds, stats if flags & nat.BN_TRAIN else None)
            rows_a = np.ascontiguousarray(rows, dtype=np.int64)
            sizes_a = np.ascontiguousarray(sizes, dtype=np.int32)
            nat.check(nat.lib().redcliff_train_steps(ctypes.byref(a), len(rows_a),
                                                     rows_a.ctypes.data_as(ctypes.c_void_p),
                                                     sizes_a.ctypes.data_as(ctypes.c_void_p), 2 * self.engines[0].F,
                                                     _stream()), "packed train_steps")
            for e in self.engines:
                e._after(flags, nbn, len(rows_a))
                e.supports_fresh = False  # the single-fit workspace's supports are stale now

    def run_epoch(self, epoch, ds):
        """The batch_update phase of `epoch` (...withStateSmoothing.py:741-759) over every batch
        of `ds`, for all replicas.  All replicas must be in the same phase."""
        kinds = [tuple(phase_of_epoch(m, epoch)) for m in self.models]
        if len(set(kinds)) != 1:
            raise RuntimeError("replicas are in different training phases at epoch %d: %s" % (epoch, kinds))
        kinds = list(kinds[0])
        if len(kinds) <= 1:
            self.run_steps(kinds, ds)
        else:  # several updates per batch: batch-major order as in batch_update
            for bi, (r, s) in enumerate(zip(ds["rows"], ds["sizes"])):
                for kind in kinds:
                    self.run_steps([kind], ds, [r], [s], ds["stats"][bi:bi + 1])
        for m in self.models:
            m._set_module_modes(kinds[-1] if kinds else None)

    def validate(self, ds):
        """validate_training loss averages (:1650-1790) of every replica: array [R][7]
        (forecast, factor, cos, fw_l1, smooth, adj, combo), plus confusion matrices [R][nsup][nsup]."""
        for e in self.engines:
            e.ensure_bound()
        self.acc.zero_()
        self.conf.zero_()
        e0 = self.engines[0]
        d = self._workspace(max(int(ds["Bmax"]), 1), ds["T"])
        flags = nat.VALUES | (nat.CONFUSION if e0.nsup > 0 else 0)
        a = self._args(d, flags, 0, ds, None)
        rows_a = np.ascontiguousarray(ds["rows"], dtype=np.int64)
        sizes_a = np.ascontiguousarray(ds["sizes"], dtype=np.int32)
        nat.check(nat.lib().redcliff_train_steps(ctypes.byref(a), len(rows_a), rows_a.ctypes.data_as(ctypes.c_void_p),
                                                 sizes_a.ctypes.data_as(ctypes.c_void_p), 2 * e0.F, _stream()),
                  "packed validate")
        acc = self.acc.cpu().numpy()
        nb = np.maximum(acc[:, 7:8], 1.0)
        ns = max(e0.nsup, 1)
        return acc[:, :7] / nb, self.conf.cpu().numpy().reshape(self.R, ns, ns)
