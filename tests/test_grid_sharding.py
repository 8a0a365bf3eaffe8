"""Host logic of packing and sharding the reference's grid searches (CPU only):

* ``shard_grid`` round-robin (the reference's SLURM task mapping, train/...gsSmooth1.py:157-160) and
  class-aware (whole shape classes per GPU, equal cost per GPU) over the reference's two grids:
  the TST grid (1536 points, 6 shape classes: embed_lag x graph-conv layers,
  train/REDCLIFF_S_CMLP_tst100hzRerun1024AvgReg_gsSmooth1.py:278-309) and the synthetic grid (990
  data sets, 25 (K, p) classes, train/REDCLIFF_S_CMLP_synSysInnovGauss1030_BSCgsSmooth3Parsim.py:140-1131);
* ``grid_packs``: one pack per shape class (mixed phase schedules allowed), sized evenly under
  max_replicas, an extra data key splitting classes.
"""
import itertools
import random

import numpy as np
import pytest
import torch

import redcliff_amd
from redcliff_amd.replicas import grid_packs, model_shape, shard_grid


def tst_grid():
    """The TST grid's points in itertools.product order (the reference's order before its shuffle):
    only the axes that change a shape or a schedule are materialised, the 8 coefficient / lr
    combinations of each are enumerated."""
    axes = dict(gen_lr=[5e-4, 1e-4], forecast=[10.0, 1.0], cos=[10.0, 1.0], smooth=[25.0, 0.025], adj=[0.1, 0.01],
                pre=[100, 50], acc=[15, 100], layers=[2, 3], lag=[16, 32, 64], embed_lr=[5e-4, 1e-4])
    keys = list(axes)
    return [dict(zip(keys, v)) for v in itertools.product(*axes.values())]


def synthetic_grid():
    """(K, p) of the 990 data sets of the synthetic grid, counts as in the reference driver."""
    counts = {(1, 3): 30, (1, 6): 105, (1, 12): 90, (2, 3): 30, (2, 6): 90, (2, 12): 90, (3, 3): 15, (3, 6): 60,
              (3, 12): 60, (4, 3): 15, (4, 6): 45, (4, 12): 45, (5, 3): 15, (5, 6): 30, (5, 12): 45, (6, 6): 30,
              (6, 12): 30, (7, 6): 15, (7, 12): 30, (8, 6): 15, (8, 12): 30, (9, 6): 15, (9, 12): 30, (10, 6): 15,
              (10, 12): 15}
    return [kp for kp, n in counts.items() for _ in range(n)]


def test_round_robin_is_the_slurm_mapping():
    assert shard_grid(10, 4, 1) == [1, 5, 9]
    assert sorted(sum((shard_grid(10, 4, r) for r in range(4)), [])) == list(range(10))


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_tst_grid_class_aware_shards(world):
    pts = tst_grid()
    assert len(pts) == 1536
    classes = [(p["lag"], p["layers"]) for p in pts]
    assert len(set(classes)) == 6
    shards = [shard_grid(len(pts), world, r, classes=classes) for r in range(world)]
    assert sorted(sum(shards, [])) == list(range(len(pts)))  # a partition
    sizes = [len(s) for s in shards]
    assert max(sizes) - min(sizes) <= 1
    for s in shards:
        # contiguous in class order: at most ceil(6 / world) + 1 classes per GPU
        assert len(set(classes[i] for i in s)) <= -(-6 // world) + 1
    # round-robin over the reference's shuffled task order (random.Random(0).shuffle, :72) puts every
    # class on every GPU
    order = list(range(len(pts)))
    random.Random(0).shuffle(order)
    rr = [[order[i] for i in shard_grid(len(pts), world, r)] for r in range(world)]
    assert all(len(set(classes[i] for i in s)) == 6 for s in rr)


def test_synthetic_grid_class_aware_shards_balance_cost():
    kp = synthetic_grid()
    assert len(kp) == 990
    cost = [k * p * p for k, p in kp]  # factor-network work of one fit ~ K p^2 (h, lags fixed)
    world = 8
    shards = [shard_grid(len(kp), world, r, classes=kp, cost=cost) for r in range(world)]
    assert sorted(sum(shards, [])) == list(range(len(kp)))
    loads = [sum(cost[i] for i in s) for s in shards]
    assert max(loads) <= 1.1 * np.mean(loads) + max(cost)
    for s in shards:
        cls = [kp[i] for i in s]
        # classes appear as contiguous runs (sorted by class order), never interleaved
        runs = [c for j, c in enumerate(cls) if j == 0 or c != cls[j - 1]]
        assert len(runs) == len(set(runs))


@pytest.mark.parametrize("grid", ["tst", "synthetic"])
def test_min_piece_merges_class_fragments(grid):
    """min_piece: no GPU keeps a sliver of a class (a pack of a few fits) -- every class piece is at
    least min(32, half the class) -- and the shares still partition the grid in class runs."""
    if grid == "tst":
        pts = tst_grid()
        classes = [(p["lag"], p["layers"]) for p in pts]
        cost = [{16: 1.3, 32: 1.55, 64: 2.03}[c[0]] + (0.2 if c[1] == 3 else 0.0) for c in classes]
    else:
        classes = synthetic_grid()
        cost = [100 * k * p * p + 11200 * p for k, p in classes]
    n, world = len(classes), 8
    plain = [shard_grid(n, world, r, classes=classes, cost=cost) for r in range(world)]
    shards = [shard_grid(n, world, r, classes=classes, cost=cost, min_piece=32) for r in range(world)]
    assert sorted(sum(shards, [])) == list(range(n))
    size = {c: classes.count(c) for c in set(classes)}
    for s in shards:
        for c in set(classes[i] for i in s):
            assert sum(1 for i in s if classes[i] == c) >= min(32, size[c] / 2.0)
        cls = [classes[i] for i in s]
        runs = [c for j, c in enumerate(cls) if j == 0 or c != cls[j - 1]]
        assert len(runs) == len(set(runs))
    # fewer packs overall than the plain cost cut, which leaves slivers on this grid
    npk = lambda sh: sum(len(set(classes[i] for i in s)) for s in sh)  # noqa: E731
    assert npk(shards) < npk(plain)


def _model(p=10, K=4, lag=20, layers=2, pre=1, acc=1):
    coeff = {"FORECAST_COEFF": 10., "FACTOR_SCORE_COEFF": 100.0, "FACTOR_COS_SIM_COEFF": 1.0,
             "FACTOR_WEIGHT_L1_COEFF": 1e-3, "FACTOR_WEIGHT_SMOOTHING_PENALTY_COEFF": 0.0, "ADJ_L1_REG_COEFF": 0.1,
             "DAGNESS_REG_COEFF": 0.0, "DAGNESS_LAG_COEFF": 0.0, "DAGNESS_NODE_COEFF": 0.0}
    eargs = [("num_features_per_node", lag), ("num_graph_conv_layers", layers), ("num_hidden_nodes", 30),
             ("sigmoid_eccentricity_coeff", 10.0)]
    torch.manual_seed(0)
    return redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing(
        p, 4, [25], lag, [0], 4, 1, K, K, coeff, False, "DGCNN", eargs, "conditional_factor_fixed_embedder",
        "apply_factor_weights_after_sim_completion", num_sims=1,
        training_mode="pretrain_embedder_then_acclimate_factors_then_combined", num_pretrain_epochs=pre,
        num_acclimation_epochs=acc)


def test_grid_packs_one_pack_per_shape_class_with_mixed_schedules():
    pts = [(lag, layers, pre, acc) for lag in (16, 32) for layers in (2, 3) for pre in (5, 10) for acc in (1, 2)]
    models = [(_model(lag=lag, layers=layers, pre=pre, acc=acc), ("oA", "oB")) for lag, layers, pre, acc in pts]
    packs = grid_packs(models)
    assert len(packs) == 4  # 2 lags x 2 layer counts; the 4 schedules share each pack
    for ms, opts, idx in packs:
        assert len(ms) == 4 and len(set(model_shape(m) for m in ms)) == 1
        assert len(set((m.num_pretrain_epochs, m.num_acclimation_epochs) for m in ms)) == 4
        assert [models[i][0] for i in idx] == ms and all(o == ("oA", "oB") for o in opts)
    # max_replicas splits a class evenly; a data key splits classes further
    assert [len(p[0]) for p in grid_packs(models, max_replicas=3)] == [2, 2] * 4
    assert len(grid_packs(models, key=lambda i: pts[i][2])) == 8
    with pytest.raises(ValueError):
        grid_packs(models, max_replicas=257)


@pytest.mark.parametrize("grid", ["tst", "synthetic"])
def test_minmax_runs_with_piece_cost(grid):
    """shard_grid(piece_cost=...): the 8 shares are contiguous runs of the class-ordered points (a
    partition; classes never interleaved inside a share) whose largest modelled cost -- points' costs
    plus piece_cost per class a share touches -- is no larger than the equal-cost cut's, and a
    bisection bound: no feasible cut has a max more than 1e-6 relative below it (checked by refilling
    at 0.999 x the bound and failing)."""
    from redcliff_amd.replicas import _minmax_runs
    if grid == "tst":
        pts = tst_grid()
        keys = [(q["lag"], q["layers"]) for q in pts]
        w = [1.0 + q["lag"] * q["layers"] / 16.0 for q in pts]
    else:
        keys = synthetic_grid()
        w = [0.5 + k * p / 12.0 for k, p in keys]
    pc = 40.0
    world = 8
    shards = [shard_grid(len(keys), world, r, classes=keys, cost=w, piece_cost=pc) for r in range(world)]
    assert sorted(sum(shards, [])) == list(range(len(keys)))

    def load(s):
        return sum(w[i] for i in s) + pc * len(set(keys[i] for i in s))
    new_max = max(load(s) for s in shards)
    old = [shard_grid(len(keys), world, r, classes=keys, cost=w) for r in range(world)]
    assert new_max <= max(load(s) for s in old) + 1e-9
    # every share is one contiguous run of the class-ordered points
    first = {}
    for c in keys:
        first.setdefault(c, len(first))
    order = sorted(range(len(keys)), key=lambda i: (first[keys[i]], i))
    pos = dict((i, j) for j, i in enumerate(order))
    for s in shards:
        js = sorted(pos[i] for i in s)
        assert js == list(range(js[0], js[0] + len(js)))
    # optimality of the bound: the class-ordered sequence cannot be cut into 8 runs under 0.999 x it
    wo = np.asarray([w[i] for i in order])
    ko = [keys[i] for i in order]
    g, cur, last, ok = 0, 0.0, None, True
    bound = 0.999 * new_max
    for j in range(len(wo)):
        add = wo[j] + (pc if ko[j] != last else 0.0)
        if cur > 0 and cur + add > bound:
            g, cur, last = g + 1, 0.0, None
            add = wo[j] + pc
        cur += add
        last = ko[j]
    assert g >= world, "a cut under 0.999 x the returned max exists"
    assert _minmax_runs(wo, ko, 1, pc).max() == 0
