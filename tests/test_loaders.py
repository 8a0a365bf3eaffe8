"""DREAM4 / LFP subset-directory data sets (redcliff_amd.data.NormalizedRecordingDirectory)
against the reference's data/dream4_datasets.py NormalizedDREAM4Dataset and
data/local_field_potential_datasets.py NormalizedLocalFieldPotentialDataset
(tests/golden/loaders.npz, written by tests/golden/make_loader_golden.py from the reference
itself).  Bar: BIT-EXACT statistics, kept order, normalised items, for the same directory
listing; file filters, NaN skipping, region averaging and the grid-search tenth included."""
import json
import os
import pickle
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))

from redcliff_amd import data as RD  # noqa: E402

G = np.load(os.path.join(HERE, "golden", "loaders.npz"))
REGIONS = json.loads(str(G["regions"]))


def rebuild(tmp, prefix):
    """Write the recordings the generator wrote (same file names, same sample order)."""
    names = sorted(set(k.split("/")[2] for k in G.files if k.startswith(prefix + "/file/")))
    for n in names:
        xs, ys = G["%s/file/%s/x" % (prefix, n)], G["%s/file/%s/y" % (prefix, n)]
        with open(os.path.join(tmp, n), "wb") as fh:
            pickle.dump([(x, y) for x, y in zip(xs, ys)], fh)


def check(tag, ds):
    listing = [str(x) for x in G[tag + "/listing"]]
    names = [n for n in listing if n in [os.path.basename(f) for f in ds.files]]
    assert np.array_equal(ds.channel_means, G[tag + "/means"])
    assert np.array_equal(ds.channel_std_devs.numpy(), G[tag + "/stds"])
    order = np.array([[names.index(os.path.basename(ds.source(i)[0])), ds.source(i)[1]] for i in range(len(ds))])
    assert np.array_equal(order.reshape(-1, 2), G[tag + "/order"].reshape(-1, 2))
    for i in range(G[tag + "/x"].shape[0]):
        x, y = ds[i]
        assert x.dtype == torch.float32 and y.dtype == torch.float32
        assert np.array_equal(x.numpy(), G[tag + "/x"][i])
        assert np.array_equal(y.numpy(), G[tag + "/y"][i])
    X, Y = ds.materialize()
    assert np.array_equal(X[:G[tag + "/x"].shape[0]].numpy(), G[tag + "/x"])


def test_dream4_directory_matches_reference(tmp_path):
    rebuild(str(tmp_path), "d4")
    listing = [str(x) for x in G["d4/listing"]]
    ds = RD.NormalizedRecordingDirectory(str(tmp_path), "dream4", shuffle=True, shuffle_seed=0, file_order=listing)
    assert len(ds) == 11  # 12 recordings, one NaN; DREAM4 has no grid-search cut
    check("d4", ds)


@pytest.mark.parametrize("tag,amap,gs", [("lfp", None, False), ("lfp_avg", REGIONS, False),
                                         ("lfp_avg_gs", REGIONS, True)])
def test_lfp_directory_matches_reference(tmp_path, tag, amap, gs):
    rebuild(str(tmp_path), "lfp")
    listing = [str(x) for x in G["lfp/listing"]]
    ds = RD.NormalizedRecordingDirectory(str(tmp_path), "lfp", shuffle=True, shuffle_seed=3, grid_search=gs,
                                         average_region_map=amap, file_order=listing)
    assert len(ds) == (2 if gs else 24)  # 25 recordings, one NaN; the grid-search tenth
    if amap is not None:
        assert ds.num_chans == len(amap)
    check(tag, ds)


def test_region_average_is_the_channel_mean():
    x = np.random.RandomState(0).randn(7, 6)
    r = RD.average_regions(x, REGIONS)
    assert r.shape == (7, 3) and r.dtype == np.float64
    assert np.array_equal(r[:, 2], np.mean(x[:, [3, 4, 5]], axis=1))


def test_train_validation_split_and_device_batches(tmp_path):
    rebuild(str(tmp_path), "d4")
    train, val = RD.load_normalized_DREAM4_data_train_test_split(str(tmp_path), 4, train_portion=0.67,
                                                                 grid_search=False)
    assert os.path.isdir(tmp_path / "train") and os.path.isdir(tmp_path / "validation")
    n_tr = sum(b[0].shape[0] for b in train)
    n_va = sum(b[0].shape[0] for b in val)
    assert n_tr + n_va == 11 and n_va > 0
    assert all(b[0].shape[1:] == (21, 10) for b in train + val)


def test_unknown_kind_and_formats_raise(tmp_path):
    with pytest.raises(ValueError):
        RD.NormalizedRecordingDirectory(str(tmp_path), "eeg")
    with pytest.raises(NotImplementedError):
        RD.NormalizedRecordingDirectory(str(tmp_path), "dream4", signal_format="directed_spectrum")
    with pytest.raises(ValueError):
        RD.NormalizedRecordingDirectory(str(tmp_path), "dream4", average_region_map=REGIONS)
