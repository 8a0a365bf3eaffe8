"""Data-parallel fit (redcliff_amd.DataParallelFit, SURVEY.md 8(e) / BASELINE configs[3]) on the
GPU: two ranks (gloo, both on cuda:0 -- the box has one GPU; the product uses RCCL) each
run the fused step on their shard in gradient-only mode, all-reduce the flat gradient and
apply the replicated Adam.  Both ranks must end bit-identical, and equal the single-device
full-batch fused fit within fp32 re-association of the gradient sum."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd")
# TST-shaped (configs[3]) with smaller batches: p=12, L=4, K=9 (3 supervised), h=25, DGCNN 16/3/100
CFG = dict(p=12, L=4, K=9, nsup=3, h=25, F=16, n=3, H=100, T=40, B=48, N=48 * 2 + 20)
EPOCHS = (0, 1, 2, 3)  # pretrain-embedder, acclimate, combined, combined


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _model():
    import redcliff_amd
    c = CFG
    K, p = c["K"], c["p"]
    coeff = {"FORECAST_COEFF": 10.0, "FACTOR_SCORE_COEFF": 100.0, "FACTOR_COS_SIM_COEFF": 1.0 / sum(range(1, K)),
             "FACTOR_WEIGHT_L1_COEFF": 1e-3, "FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF": 0.0,
             "ADJ_L1_REG_COEFF": 0.1 / K / np.sqrt(p * p - 1.0), "DAGNESS_REG_COEFF": 0.0, "DAGNESS_LAG_COEFF": 0.0,
             "DAGNESS_NODE_COEFF": 0.0}
    eargs = [("num_features_per_node", c["F"]), ("num_graph_conv_layers", c["n"]), ("num_hidden_nodes", c["H"]),
             ("sigmoid_eccentricity_coeff", 10.0)]
    torch.manual_seed(0)
    m = redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing(
        p, c["L"], [c["h"]], c["F"], [0], c["L"], 1, K, c["nsup"], coeff, False, "DGCNN", eargs,
        "conditional_factor_fixed_embedder", "apply_factor_weights_after_sim_completion", num_sims=1,
        training_mode="pretrain_embedder_then_acclimate_factors_then_combined", num_pretrain_epochs=1,
        num_acclimation_epochs=1).cuda()
    oA = torch.optim.Adam(m.gen_model[0].parameters(), lr=5e-4, betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    oB = torch.optim.Adam(m.gen_model[1].parameters(), lr=5e-4, betas=(0.9, 0.999), eps=1e-4, weight_decay=1e-4)
    return m, oA, oB


def _loader():
    c = CFG
    rng = np.random.RandomState(7)
    X = rng.randn(c["N"], c["T"], c["p"]).astype(np.float32)
    for t in range(2, c["T"]):
        X[:, t] += 0.4 * X[:, t - 1] - 0.2 * X[:, t - 2]
    Y = np.zeros((c["N"], c["K"], c["T"]), np.float32)
    Y[np.arange(c["N"]), rng.randint(0, c["K"], c["N"]), :] = 1.0
    X, Y = torch.from_numpy(X), torch.from_numpy(Y)
    return [(X[i:i + c["B"]], Y[i:i + c["B"]]) for i in range(0, c["N"], c["B"])]


def _worker(rank, world, port, outdir, sharded=True):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from redcliff_amd import DataParallelFit
    m, oA, oB = _model()
    dp = DataParallelFit(m, oA, oB)
    ds = dp.cache_dataset(_loader(), sharded=sharded)
    if sharded:  # only this rank's windows are resident; the whole batches it uploaded are its own
        assert ds["X"].shape[0] == int(ds["local_sizes"].sum()) < CFG["N"]
        assert dp.uploaded_windows < CFG["N"]
    for epoch in EPOCHS:
        dp.run_epoch(epoch, ds)
    conf = dp.train_confusion()
    torch.cuda.synchronize()
    sd = dict((k, v.detach().cpu()) for k, v in m.state_dict().items())
    torch.save({"state": sd, "conf": torch.from_numpy(conf)}, os.path.join(outdir, "rank%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_data_parallel_matches_full_batch(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, start_method="spawn",
                       join=True)
    r0 = torch.load(str(tmp_path / "rank0.pt"), weights_only=True)
    r1 = torch.load(str(tmp_path / "rank1.pt"), weights_only=True)
    for k in r0["state"]:
        np.testing.assert_array_equal(r0["state"][k].numpy(), r1["state"][k].numpy(), err_msg="ranks differ: " + k)
    # single-device, full-batch fused fit of the same model on the same batches
    m, oA, oB = _model()
    loader = _loader()
    eng = m.engine()
    ds = eng.cache_dataset(loader)
    for epoch in EPOCHS:
        eng.conf.zero_()
        for bi, (Xb, Yb) in enumerate(loader):
            m.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
    conf = eng.conf.cpu().numpy().reshape(CFG["nsup"], CFG["nsup"])  # last epoch's counts
    del ds
    want = m.state_dict()
    for k, v in want.items():
        got = r0["state"][k].numpy().astype(np.float64)
        w = v.detach().cpu().numpy().astype(np.float64)
        if k.endswith("num_batches_tracked"):
            assert int(got) == int(w), k
            continue
        tol = 5e-6 * max(1.0, np.abs(w).max()) + 2e-4 * np.abs(w)
        bad = np.abs(got - w) > tol
        assert not bad.any(), "%s: %d/%d off, max err %.3e" % (k, int(bad.sum()), w.size, np.abs(got - w).max())
    np.testing.assert_array_equal(r0["conf"].numpy(), conf)


def test_sharded_cache_bitwise_equals_whole_set(tmp_path):
    """DataParallelFit.cache_dataset keeps only the rank's shard windows resident (their rows
    renumbered, the global batches' BatchNorm statistics taken from the whole batch by the same
    kernel): both ranks end bit-identical to the run with the whole set on every rank."""
    world = 2
    for sharded in (True, False):
        out = tmp_path / ("s%d" % int(sharded))
        out.mkdir()
        mp.start_processes(_worker, args=(world, _free_port(), str(out), sharded), nprocs=world,
                           start_method="spawn", join=True)
    for r in range(world):
        a = torch.load(str(tmp_path / "s1" / ("rank%d.pt" % r)), weights_only=True)
        b = torch.load(str(tmp_path / "s0" / ("rank%d.pt" % r)), weights_only=True)
        for k in b["state"]:
            np.testing.assert_array_equal(a["state"][k].numpy(), b["state"][k].numpy(), err_msg="rank %d %s" % (r, k))
        np.testing.assert_array_equal(a["conf"].numpy(), b["conf"].numpy())


def test_large_shard_takes_the_matrix_core_factor_path(monkeypatch):
    """512 windows per step at the TST shape exceed the vector factor backward's 64 KiB LDS
    budget (it stages per-window terms of the whole batch); the step then runs the matrix-core
    factor path instead of failing -- the same bits as forcing that path."""
    c = CFG
    rng = np.random.RandomState(3)
    X = torch.from_numpy(rng.randn(512, c["T"], c["p"]).astype(np.float32))
    Y = torch.zeros(512, c["K"], c["T"])
    Y[torch.arange(512), torch.from_numpy(rng.randint(0, c["K"], 512))] = 1.0
    out = []
    for path in (None, "mfma"):
        if path is None:
            monkeypatch.delenv("REDCLIFF_FAC_PATH", raising=False)
        else:
            monkeypatch.setenv("REDCLIFF_FAC_PATH", path)
        m, oA, oB = _model()
        for ep in (0, 1, 2):  # pretrain, acclimate, combined
            m.batch_update(ep, 0, X, Y, oA, oB, 1)
        torch.cuda.synchronize()
        out.append(dict((k, v.detach().cpu().numpy()) for k, v in m.state_dict().items()))
    for k in out[0]:
        np.testing.assert_array_equal(out[0][k], out[1][k], err_msg=k)


FIT_KW = dict(lookback=1, check_every=1, verbose=0, stopping_criteria_forecast_coeff=10.,
              stopping_criteria_factor_coeff=100., stopping_criteria_cosSim_coeff=1.)
FIT_EPOCHS = 7


def _val_loader():
    c = CFG
    rng = np.random.RandomState(8)
    X = rng.randn(40, c["T"], c["p"]).astype(np.float32)
    Y = np.zeros((40, c["K"], c["T"]), np.float32)
    Y[np.arange(40), rng.randint(0, c["K"], 40), :] = 1.0
    X, Y = torch.from_numpy(X), torch.from_numpy(Y)
    return [(X[i:i + 24], Y[i:i + 24]) for i in range(0, 40, 24)]


def _true_gc():
    rng = np.random.RandomState(9)
    return [(rng.rand(CFG["p"], CFG["p"], CFG["L"]) < 0.25).astype(np.float64) for _ in range(CFG["nsup"])]


def _fit_worker(rank, world, port, outdir):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from redcliff_amd import DataParallelFit
    m, oA, oB = _model()
    dp = DataParallelFit(m, oA, oB)
    save = os.path.join(outdir, "ckpt%d" % rank)
    train = _loader()
    ret = dp.fit(save, train, 1, FIT_EPOCHS, _val_loader(), GC=_true_gc(), **FIT_KW)
    torch.cuda.synchronize()
    # the fit trained from the rank's shard cache: the engine never cached the whole training set
    eng = m.engine()
    assert id(train) not in eng.dataset_cache
    assert all(int(ds_["X"].shape[0]) < CFG["N"] for ds_ in eng.dataset_cache.values())
    assert dp.uploaded_windows < CFG["N"]
    h = m.fit_history
    sd = dict((k, v.detach().cpu()) for k, v in m.state_dict().items())
    hist = dict((k, torch.tensor(np.asarray(h[k], np.float64))) for k in
                ("avg_forecasting_loss", "avg_factor_loss", "avg_factor_cos_sim_penalty", "avg_fw_l1_penalty",
                 "avg_adj_penalty", "avg_combo_loss"))
    f1 = torch.tensor(np.asarray([h["f1score_histories"][0.0][sf] for sf in range(CFG["nsup"])], np.float64))
    torch.save({"state": sd, "hist": hist, "f1": f1, "best_it": int(h["best_it"]),
                "stopped_at": -1 if h["stopped_at"] is None else int(h["stopped_at"]), "ret": float(ret),
                "files": sorted(os.listdir(save)) if os.path.isdir(save) else []},
               os.path.join(outdir, "fit%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_data_parallel_fit_matches_single_device_fit(tmp_path):
    """DataParallelFit.fit (configs[3]: a whole fit, not just epochs): two ranks (gloo, one GPU)
    vs the single-device fit() of the same model on the same batches -- loss histories within
    1e-4 relative (the sharded gradient sum re-associates fp32 additions), the same best epoch,
    stopping epoch and F1 history, final parameters within the step test's tolerance; both ranks
    bit-identical; checkpoints written by rank 0 only."""
    world = 2
    mp.start_processes(_fit_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, start_method="spawn",
                       join=True)
    r0 = torch.load(str(tmp_path / "fit0.pt"), weights_only=True)
    r1 = torch.load(str(tmp_path / "fit1.pt"), weights_only=True)
    for k in r0["state"]:
        np.testing.assert_array_equal(r0["state"][k].numpy(), r1["state"][k].numpy(), err_msg="ranks differ: " + k)
    for k in r0["hist"]:
        np.testing.assert_array_equal(r0["hist"][k].numpy(), r1["hist"][k].numpy(), err_msg=k)
    assert r0["best_it"] == r1["best_it"] and r0["stopped_at"] == r1["stopped_at"]
    assert "training_meta_data_and_hyper_parameters.pkl" in r0["files"] and r1["files"] == []
    m, oA, oB = _model()
    ret = m.fit(None, _loader(), oA, oB, CFG["L"], 1, 1, FIT_EPOCHS, _val_loader(), GC=_true_gc(), **FIT_KW)
    h = m.fit_history
    for k, v in r0["hist"].items():
        w = np.asarray(h[k], np.float64)
        assert v.numpy().shape == w.shape, k
        np.testing.assert_allclose(v.numpy(), w, rtol=1e-4, atol=1e-6, err_msg=k)
    assert r0["best_it"] == h["best_it"]
    assert r0["stopped_at"] == (-1 if h["stopped_at"] is None else h["stopped_at"])
    f1 = np.asarray([h["f1score_histories"][0.0][sf] for sf in range(CFG["nsup"])], np.float64)
    np.testing.assert_allclose(r0["f1"].numpy(), f1, rtol=0, atol=1e-6)
    np.testing.assert_allclose(r0["ret"], ret, rtol=1e-4)
    for k, v in m.state_dict().items():
        got = r0["state"][k].numpy().astype(np.float64)
        w = v.detach().cpu().numpy().astype(np.float64)
        if k.endswith("num_batches_tracked"):
            assert int(got) == int(w), k
            continue
        tol = 5e-6 * max(1.0, np.abs(w).max()) + 2e-4 * np.abs(w)
        bad = np.abs(got - w) > tol
        assert not bad.any(), "%s: %d/%d off, max err %.3e" % (k, int(bad.sum()), w.size, np.abs(got - w).max())


def test_fused_update_bitwise_equals_per_group_adam(monkeypatch):
    """redcliff_dp_update (Adam of both groups + the supports of the new A, one launch) against
    the per-group redcliff_adam_apply sequence with the supports refreshed by the next step:
    one rank (gloo), the same batches, bit for bit after every epoch of the schedule."""
    import torch.distributed as dist
    from redcliff_amd import DataParallelFit
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        runs = {}
        for fused in (False, True):
            m, oA, oB = _model()
            dp = DataParallelFit(m, oA, oB, fused_update=fused)
            ds = dp.cache_dataset(_loader())
            hist = []
            for epoch in EPOCHS:
                dp.run_epoch(epoch, ds)
                torch.cuda.synchronize()
                hist.append({k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()})
            runs[fused] = hist
    finally:
        dist.destroy_process_group()
    for e, (want, got) in enumerate(zip(runs[False], runs[True])):
        for k, w in want.items():
            np.testing.assert_array_equal(got[k], w, err_msg="epoch %d: %s" % (EPOCHS[e], k))
