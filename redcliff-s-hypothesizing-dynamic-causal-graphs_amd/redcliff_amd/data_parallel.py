"""Data-parallel REDCLIFF-S fitting for large recordings (BASELINE configs[3]).

The reference fits one model per process (no torch.distributed anywhere).  For the LFP
recordings (TST, many windows per subject) one fit is spread over the GPUs of a node:

  * every rank holds the same model (parameters broadcast from rank 0 at construction) and, in
    device memory, only the windows of its own shards of the training set (cache_dataset: a global
    batch is uploaded whole by one owner rank, which takes its BatchNorm statistics; the others
    upload their shards and receive the statistics in one all-reduce of the [nbatch][2][F] table);
  * each global batch of B windows is split into world_size contiguous shards; rank g runs
    the fused step on its shard in gradient-only mode (RC_GRAD_ONLY) with B_global = B, so
    batch-mean terms (forecast MSE :629, factor MSE :638-661) are scaled by 1/B and batch
    sums (fw-L1 :666, adj-L1 :696-715) are not: the shard gradients sum to the full-batch
    gradient.  The cos-sim penalty carries no gradient (metrics.py:380);
  * BatchNorm uses the statistics of the GLOBAL batch (computed once per batch, at caching time,
    from the whole batch by its owner rank with the same kernel as the single fit's), so no SyncBN
    collective runs per step and the running statistics advance identically on every rank;
  * one all-reduce (sum) of one flat fp32 gradient buffer per update (embedder + factor
    groups, 0.4-0.9 MB at the published configs) over RCCL / xGMI, then the replicated Adam
    update of both groups in one launch (redcliff_dp_update, which also refreshes the DGCNN
    supports of the new A) -- every rank ends every step with identical parameters.

Works with any torch.distributed backend whose all_reduce takes device tensors ("nccl" =
RCCL on ROCm for the real thing; "gloo" for tests on one GPU).
"""
import ctypes
import os

import numpy as np
import torch
import torch.distributed as dist

from . import _native as nat
from .engine import _stream, flags_for, phase_of_epoch, select_labels
from .kernels import ptr


def shard_of(B, world, rank):
    """Contiguous shard (offset, size) of rank `rank` in a batch of B windows: sizes differ by
    at most one, the first B % world ranks take the extra window."""
    base, extra = divmod(int(B), int(world))
    size = base + (1 if rank < extra else 0)
    off = rank * base + min(rank, extra)
    return off, size


class DataParallelFit:
    """One REDCLIFF-S fit sharded over the ranks of `group` (default: the world)."""

    def __init__(self, model, optimizerA, optimizerB, group=None, fused_update=None):
        if not dist.is_initialized():
            raise RuntimeError("DataParallelFit needs torch.distributed.init_process_group first")
        self.model = model
        self.oA, self.oB = optimizerA, optimizerB
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.eng = eng = model.engine()
        eng.ensure_bound()
        eng.bind_optimizer("A", optimizerA)
        eng.bind_optimizer("B", optimizerB)
        # identical starting point on every rank (rank 0's parameters and BN buffers)
        src = dist.get_global_rank(group, 0) if group is not None else 0
        for t in (eng.emb, eng.fac, eng.bn):
            dist.broadcast(t, src, group=group)
        eng.invalidate()
        self.PA, self.PB = eng.emb.numel(), eng.fac.numel()
        self.grad = torch.zeros(self.PA + self.PB, device=eng.device, dtype=torch.float32)
        self.gE, self.gF = self.grad[:self.PA], self.grad[self.PA:]
        self.comm_bytes = 0
        self._bn_pending = 0
        # fused_update: Adam of both groups + the supports refresh in one launch (redcliff_dp_update);
        # False: one redcliff_adam_apply per group, supports refreshed by the next step (the
        # round-2 sequence, kept as the check of the fused launch)
        if fused_update is None:
            fused_update = os.environ.get("REDCLIFF_DP_FUSED", "1") != "0"
        self.fused_update = bool(fused_update)

    def cache_dataset(self, loader, sharded=None):
        """The training set on the device.  sharded (default; REDCLIFF_DP_SHARDED=0 or
        sharded=False keeps the whole set on every rank, the round-4 layout): each global batch of
        the loader goes to the device ONCE over the whole group: global batch bi is uploaded whole
        only by its owner rank (bi mod world), which takes its BatchNorm batch statistics from the
        whole batch (k_bn_stats, one workgroup per feature in a fixed order: the bits of the
        whole-set cache); every other rank uploads only its own shard of it (shard_of).  The 2 F
        doubles per batch reach the other ranks in ONE all-reduce over the [nbatch][2][F] table
        (each row is non-zero on its owner only, so the sum is exact), and only this rank's shards
        stay resident -- 1 / world of the windows."""
        if sharded is None:
            sharded = os.environ.get("REDCLIFF_DP_SHARDED", "1") != "0"
        if not sharded:
            return self.eng.cache_dataset(loader)
        cache = self.__dict__.setdefault("_shard_cache", {})
        if id(loader) in cache:
            return cache[id(loader)]
        eng = self.eng
        xs, ls, sizes, local, stats = [], [], [], [], []
        T = None
        for bi, (X, Y) in enumerate(loader):
            B = int(X.shape[0])
            off, Bl = shard_of(B, self.world, self.rank)
            if Bl < 1:
                raise ValueError("batch %d has %d windows for %d ranks: every rank needs at least one window"
                                 % (bi, B, self.world))
            T = int(X.shape[1])
            if bi % self.world == self.rank:  # the batch's owner: the whole batch, for its statistics
                Xd = X.to(eng.device, torch.float32).contiguous()
                stats.append(eng.bn_stats(eng.dims(1, T), Xd, B, B))
                xs.append(Xd[off:off + Bl].clone())
            else:
                Xd = None
                stats.append(torch.zeros(1, 2, eng.F, device=eng.device, dtype=torch.float64))
                xs.append(X[off:off + Bl].to(eng.device, torch.float32).contiguous())
            lab = select_labels(Y, eng.K, eng.Lmax) if Y is not None else torch.zeros(B, eng.K)
            ls.append(lab[off:off + Bl].to(eng.device, torch.float32))
            sizes.append(B)
            local.append(Bl)
            del Xd
        rows = np.cumsum([0] + local[:-1]).astype(np.int64)  # the rank's rows of each batch in its X
        stats = torch.cat(stats, 0).contiguous()
        if self.world > 1:
            dist.all_reduce(stats, op=dist.ReduceOp.SUM, group=self.group)
        self.uploaded_windows = int(sum(s_ if bi % self.world == self.rank else l_
                                        for bi, (s_, l_) in enumerate(zip(sizes, local))))
        ds = {"X": torch.cat(xs, 0).contiguous(), "lab": torch.cat(ls, 0).contiguous(), "rows": rows,
              "sizes": np.asarray(sizes, dtype=np.int32), "local_sizes": np.asarray(local, dtype=np.int32),
              "stats": stats, "T": T, "Bmax": max(sizes), "len": len(sizes),
              "loader": loader, "sharded": True}
        cache[id(loader)] = ds
        return ds

    def _step(self, kind, ds, bi):
        eng = self.eng
        flags, nbn = flags_for(kind, eng.nsup)
        stepA, stepB = bool(flags & nat.STEP_A), bool(flags & nat.STEP_B)
        B = int(ds["sizes"][bi])
        off, Bl = shard_of(B, self.world, self.rank)
        if Bl < 1:
            raise ValueError("batch %d has %d windows for %d ranks: every rank needs at least one window"
                             % (bi, B, self.world))
        d = eng.workspace(-(-int(ds["Bmax"]) // self.world), ds["T"])  # the largest shard
        stats = ds["stats"][bi:bi + 1] if flags & nat.BN_TRAIN else None
        a = eng._args(d, flags | nat.GRAD_ONLY, nbn, ds["X"], ds["lab"], stats)
        # the rank's rows: in its own shard cache, or at `off` inside the batch of a whole-set cache
        a.row0 = int(ds["rows"][bi]) + (0 if ds.get("sharded") else off)
        a.B = Bl
        a.B_global = B
        a.grad_emb, a.grad_fac = ptr(self.gE), ptr(self.gF)
        nat.check(nat.lib().redcliff_train_step(ctypes.byref(a), _stream()), "data-parallel shard step")
        # one collective per update: the stepped groups' gradients, summed over ranks
        buf = self.grad if (stepA and stepB) else (self.gE if stepA else self.gF)
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)
        self.comm_bytes += buf.numel() * 4
        if self.fused_update:
            # Adam of both groups from the summed gradients and the supports of the updated A, one
            # launch with the shard step's own arguments (t = tA / tB, the same hyper-parameters)
            nat.check(nat.lib().redcliff_dp_update(ctypes.byref(a), self.PA, self.PB, _stream()), "dp_update")
        else:
            hyp = eng._hyper()
            d1 = eng.dims(1, ds["T"])  # Adam over the flat groups: only R and the layouts matter
            for g, on, P, buf_g, n in (("A", stepA, eng.emb, self.gE, self.PA), ("B", stepB, eng.fac, self.gF, self.PB)):
                if on:
                    st = eng.opt[g]
                    nat.check(nat.lib().redcliff_adam_apply(ctypes.byref(d1), ptr(P), ptr(st["m"]), ptr(st["v"]),
                                                            ptr(buf_g), n, n, ptr(hyp), 0 if g == "A" else 1, st["t"] + 1,
                                                            _stream()), "adam_apply")
        # step counters (host, and the optimizers' CPU step tensors, which _args reads back to
        # detect torch-stepped optimizers); BatchNorm's num_batches_tracked, a device tensor the
        # kernels do not read, is advanced once per run (flush), not with a launch per update
        if stepA:
            eng.opt["A"]["t"] += 1
        if stepB:
            eng.opt["B"]["t"] += 1
        eng._sync_steps()
        self._bn_pending += nbn
        eng._mark_fresh()  # the fused update refreshed the supports of the new A
        if stepA and not self.fused_update:
            eng.supports_fresh = False  # A moved after the step's own support refresh

    def _flush(self):
        """The BatchNorm update count deferred by _step."""
        if self._bn_pending:
            self.eng.dgcnn.BN1.num_batches_tracked.add_(self._bn_pending)
            self._bn_pending = 0

    def run_steps(self, kind, ds, batches):
        """Updates of one kind over the global batches `batches` (indices into ds), back to back:
        everything is enqueued on the stream (the RCCL all-reduce included), the host never
        waits."""
        for bi in batches:
            self._step(kind, ds, bi)
        self._flush()

    def run_epoch(self, epoch, ds, set_modes=True):
        """The batch_update phase of `epoch` (...withStateSmoothing.py:741-759) over every global
        batch of `ds`, sharded over the ranks."""
        kinds = phase_of_epoch(self.model, epoch)
        self.eng.conf.zero_()
        for bi in range(int(ds["len"])):
            for kind in kinds:
                self._step(kind, ds, bi)
        self._flush()
        if set_modes:
            self.model._set_module_modes(kinds[-1] if kinds else None)

    def fit(self, save_dir, X_train, output_length, max_iter, X_val, lookback=5, check_every=50, verbose=1, GC=None,
            deltaConEps=0.1, in_degree_coeff=1., out_degree_coeff=1., stopping_criteria_forecast_coeff=1.,
            stopping_criteria_factor_coeff=1., stopping_criteria_cosSim_coeff=1., save_plots=False):
        """The reference's whole ``fit`` (models/redcliff_s_cmlp_withStateSmoothing.py:1175-1647)
        with every training epoch sharded over the ranks:

          * training: run_epoch (one RCCL all-reduce of the flat gradient per update), then the
            epoch's factor-score confusion matrix summed over the ranks (:786-803, :1344-1364);
          * everything after the training steps of an epoch -- GC tracking on the first
            validation batch (:1366-1414), validate_training (:1416-1480), the stopping rule
            (:1482-1559), best-model snapshots, restore_parameters (:1621) and the final
            validation -- is the single fit's device-side epoch (fit_loop._device_epochs) run
            on EVERY rank: every rank holds the same parameters (bit-identical after each
            replicated Adam step) and the same validation windows, so every rank computes the
            same values with the same fixed-order kernels and takes the same decisions without
            a collective (tests/test_gpu_data_parallel.py checks the ranks end bit-identical);
          * checkpoints and the final model file are written by rank 0 only.
        The next epoch trains speculatively while the host digests the current one, exactly as in
        the single fit (undone on every rank when the fit stops).  Returns what fit returns;
        model.fit_history holds the histories."""
        from .fit_loop import run_fit
        m = self.model
        if "Freeze" in m.training_mode or "pretrain_factor" in m.training_mode:
            raise NotImplementedError("the data-parallel fit runs the published schedule (pretrain embedder, "
                                      "acclimate, combined); got training_mode=%s" % m.training_mode)
        ds = self.cache_dataset(X_train)

        def runner(epoch):
            self.run_epoch(epoch, ds, set_modes=False)
            if self.eng.nsup > 0:
                dist.all_reduce(self.eng.conf, op=dist.ReduceOp.SUM, group=self.group)

        return run_fit(m, save_dir, X_train, self.oA, self.oB, output_length, max_iter, X_val, lookback, check_every,
                       verbose, GC, deltaConEps, in_degree_coeff, out_degree_coeff, (None, "CosineSimilarity", 0, 10),
                       stopping_criteria_forecast_coeff, stopping_criteria_factor_coeff,
                       stopping_criteria_cosSim_coeff, save_plots, runner=runner, writer=self.rank == 0,
                       train_ds=ds)

    def train_confusion(self):
        """Factor-score confusion matrix of the last epoch summed over ranks (:786-803)."""
        c = self.eng.conf.clone()
        dist.all_reduce(c, op=dist.ReduceOp.SUM, group=self.group)
        n = max(self.eng.nsup, 1)
        return c.cpu().numpy().reshape(n, n)


def global_batches(n_windows, B):
    """(rows, sizes) of consecutive global batches, as the reference DataLoader yields them."""
    rows = np.arange(0, n_windows, B, dtype=np.int64)
    sizes = np.minimum(B, n_windows - rows).astype(np.int32)
    return rows, sizes
