"""Generate tests/golden/loaders.npz from the REFERENCE's DREAM4 and LFP data sets (build
container only).

    python tests/golden/make_loader_golden.py

This script writes its OWN small subset-pickle directories (seeded random recordings in the
reference's file layout: a pickled list of (x (T, C), y) samples per ``subset_*`` /
``*_subset*`` file, plus files the filters must skip and one NaN recording), then runs
data/dream4_datasets.py NormalizedDREAM4Dataset and data/local_field_potential_datasets.py
NormalizedLocalFieldPotentialDataset (with and without a region-averaging map, with and
without the grid-search cut) on them.  Stored: the recordings, the directory listing the
reference saw, channel means / std devs, the kept (file, position) order and the first
normalised items.  Only arrays leave this script.
"""
import contextlib
import io
import json
import os
import pickle
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.ref_import import import_reference  # noqa: E402

import_reference()
import importlib  # noqa: E402

d4 = importlib.import_module("data.dream4_datasets")
lfp = importlib.import_module("data.local_field_potential_datasets")

REGIONS = {"amy": [0, 2], "hip": [1], "pfc": [3, 4, 5]}


def write_dir(tmp, files, rng, T, C, K, nan_at=None, label_T=None):
    """files: {name: n_samples}.  Returns {name: [(x, y), ...]} as written."""
    out = {}
    for fi, (name, n) in enumerate(files.items()):
        smps = []
        for j in range(n):
            x = rng.randn(T, C) * (1.0 + 0.5 * np.arange(C)) + np.arange(C)
            if nan_at == (fi, j):
                x[3, 1] = np.nan
            y = np.zeros(K) if label_T is None else np.zeros((K, label_T))
            y[rng.randint(K)] = 1.0
            smps.append((x, y))
        out[name] = smps
        with open(os.path.join(tmp, name), "wb") as fh:
            pickle.dump(smps, fh)
    return out


def record(prefix, ds, files_written, listing, out):
    names = [n for n in listing if n in files_written]
    out[prefix + "/listing"] = np.array(listing)
    out[prefix + "/means"] = np.asarray(ds.channel_means)
    out[prefix + "/stds"] = ds.channel_std_devs.numpy()
    out[prefix + "/order"] = np.array([[names.index(os.path.basename(p)), j] for p, j in ds.data])
    items = [ds[i] for i in range(min(3, len(ds)))]
    out[prefix + "/x"] = np.stack([x.numpy() for x, _ in items])
    out[prefix + "/y"] = np.stack([y.numpy() for _, y in items])


def main():
    out = {}
    rng = np.random.RandomState(21)
    # DREAM4: subset_* files; "metadata" and non-subset files skipped; one NaN recording
    with tempfile.TemporaryDirectory() as tmp:
        files = {"subset_0.pkl": 5, "subset_1.pkl": 4, "subset_2.pkl": 3}
        written = write_dir(tmp, files, rng, T=21, C=10, K=4, nan_at=(1, 2))
        write_dir(tmp, {"subset_metadata.pkl": 1, "other.pkl": 2}, rng, T=21, C=10, K=4)
        listing = os.listdir(tmp)
        with contextlib.redirect_stdout(io.StringIO()):
            ds = d4.NormalizedDREAM4Dataset(tmp, "original", shuffle=True, shuffle_seed=0)
        record("d4", ds, written, listing, out)
        for name, smps in written.items():
            out["d4/file/%s/x" % name] = np.stack([s[0] for s in smps])
            out["d4/file/%s/y" % name] = np.stack([s[1] for s in smps])
    # LFP: *_subset* files, 25 recordings (grid-search tenth = 2), per-time-step labels
    with tempfile.TemporaryDirectory() as tmp:
        files = {"mouse3_subset_0.pkl": 9, "mouse3_subset_1.pkl": 8, "mouse5_subset_0.pkl": 8}
        written = write_dir(tmp, files, rng, T=30, C=6, K=3, nan_at=(2, 5), label_T=30)
        write_dir(tmp, {"mouse3_subset_metadata.pkl": 1, "subset_9.pkl": 2}, rng, T=30, C=6, K=3, label_T=30)
        listing = os.listdir(tmp)
        for tag, amap, gs in (("lfp", None, False), ("lfp_avg", REGIONS, False), ("lfp_avg_gs", REGIONS, True)):
            with contextlib.redirect_stdout(io.StringIO()):
                ds = lfp.NormalizedLocalFieldPotentialDataset(tmp, "original", shuffle=True, shuffle_seed=3,
                                                              grid_search=gs, average_region_map=amap)
            record(tag, ds, written, listing, out)
        for name, smps in written.items():
            out["lfp/file/%s/x" % name] = np.stack([s[0] for s in smps])
            out["lfp/file/%s/y" % name] = np.stack([s[1] for s in smps])
    out["regions"] = json.dumps(REGIONS)
    np.savez_compressed(os.path.join(HERE, "loaders.npz"), **out)
    print("wrote loaders.npz (%d arrays)" % len(out))


if __name__ == "__main__":
    main()
