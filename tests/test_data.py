"""Synthetic sVAR generator and normalised window set (redcliff_amd.data) against the
reference's data/data_utils.py generate_synthetic_data and data/synthetic_datasets.py
NormalizedSyntheticWVARDataset (tests/golden/svar_data.npz, written by
tests/golden/make_data_golden.py).  Bar: BIT-EXACT recordings, labels, statistics,
order and normalised items for the same seed."""
import json
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))

from redcliff_amd import data as RD  # noqa: E402

G = np.load(os.path.join(HERE, "golden", "svar_data.npz"))
GENS = sorted(set(k.split("/")[0] for k in G.files if k.startswith("gen")))


def generate(name, rng=None):
    cfg = json.loads(str(G[name + "/meta"]))
    D, S = cfg["D"], cfg["S"]
    if rng is None:
        np.random.seed(9999)
    return RD.generate_synthetic_data(cfg["N"], cfg["T"], cfg["label"], cfg["burn"], D, S, cfg["nlab"], 2,
                                      G[name + "/A"], G[name + "/f"], G[name + "/mu"], G[name + "/var"],
                                      G[name + "/amp"], cfg["nl"], noise_type=cfg["noise"],
                                      activation_codes=G[name + "/codes"], rng=rng)


@pytest.mark.parametrize("name", GENS)
def test_generator_bit_exact(name):
    X, Y = generate(name)
    assert np.array_equal(X, G[name + "/X"]), float(np.abs(X - G[name + "/X"]).max())
    assert np.array_equal(Y, G[name + "/Y"])


def test_generator_private_rng_same_stream():
    X1, _ = generate(GENS[0])
    X2, _ = generate(GENS[0], rng=np.random.RandomState(9999))
    assert np.array_equal(X1, X2)


def test_normalized_window_set_matches_reference():
    X, Y = G["gen0/X"], G["gen0/Y"]
    ds = RD.NormalizedWindowSet(list(X), list(Y), shuffle=True, shuffle_seed=0, grid_search=False)
    assert np.array_equal(ds.channel_means, G["ds/means"])
    assert np.array_equal(ds.channel_std_devs.numpy(), G["ds/stds"])
    assert ds.data == list(G["ds/order"])
    for i in range(3):
        x, y = ds[i]
        assert x.dtype == torch.float32
        assert np.array_equal(x.numpy(), G["ds/x"][i])
        assert np.array_equal(y.numpy(), G["ds/y"][i])
    gs = RD.NormalizedWindowSet(list(X), list(Y), shuffle=True, shuffle_seed=0, grid_search=True)
    assert gs.data == list(G["ds/order_gs"])
    Xm, Ym = ds.materialize()
    assert np.array_equal(Xm[:3].numpy(), G["ds/x"])
    b = ds.batches(4)
    assert [t[0].shape[0] for t in b] == [4, len(ds) - 4]


def test_nan_recordings_are_skipped():
    X = np.random.RandomState(0).randn(8, 10, 3)
    X[2, 4, 1] = np.nan
    ds = RD.NormalizedWindowSet(list(X), [np.zeros((2, 10))] * 8, shuffle=False, grid_search=False)
    assert ds.data == [0, 1, 3, 4, 5, 6, 7]
    assert np.all(np.isfinite(ds.channel_means))
