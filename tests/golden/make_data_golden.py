"""Generate tests/golden/svar_data.npz from the REFERENCE's data code (build container only).

    python tests/golden/make_data_golden.py

* data/data_utils.py generate_synthetic_data on small seeded systems (both noise types,
  both label types, identity / min-max edge activations, more states than labels), with
  ``np.random.seed`` set first exactly as the curation script does (seed 9999,
  data/currate_sVARwInnovativeContinuousGaussianNoise_data_etNL.py:13).  Plots go to a
  temporary directory.
* data/synthetic_datasets.py NormalizedSyntheticWVARDataset over one subset file that
  THIS script writes (its own pickle of the generated samples, in a temporary
  directory): channel means / std devs, the shuffled + grid-search-cut order, and the
  first normalised items.
Only arrays are stored.
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

du = importlib.import_module("data.data_utils")
sd = importlib.import_module("data.synthetic_datasets")

ACTS = {0: None, 1: (lambda x: x), 2: (lambda x: np.min((x, 0))), 3: (lambda x: np.max((x, 0)))}


def system(rng, S, D, density=0.35):
    A = np.zeros((S, D, D, 2))
    for k in range(S):
        mask = rng.rand(D, D) < density
        A[k, :, :, 0] = mask * 0.3
        A[k, :, :, 1] = mask * 0.3 * (rng.rand(D, D) < 0.5)
        A[k, np.arange(D), np.arange(D), 0] = 0.6
        A[k, np.arange(D), np.arange(D), 1] = 1.0
    return A


CASES = [
    dict(N=6, T=20, burn=10, D=5, S=2, nlab=2, label="OneHot", noise="gaussian", nl=1.0, acts="minmax"),
    dict(N=5, T=16, burn=10, D=4, S=3, nlab=2, label="Oracle", noise="white", nl=4.0, acts="identity"),
    dict(N=4, T=12, burn=5, D=6, S=3, nlab=3, label="OneHot", noise="white", nl=0.0, acts="none"),
]


def main():
    out = {}
    rng = np.random.RandomState(11)
    for c, cfg in enumerate(CASES):
        D, S = cfg["D"], cfg["S"]
        A = system(rng, S, D)
        codes = np.zeros((S, D, D, 2), dtype=np.int64)
        if cfg["acts"] == "identity":
            codes[:] = 1
        elif cfg["acts"] == "minmax":
            codes[..., 0], codes[..., 1] = 2, 3
            codes[:, np.arange(D), np.arange(D), :] = 0
        nonlin = [[[[ACTS[int(codes[k, i, j, l])] for l in range(2)] for j in range(D)] for i in range(D)]
                  for k in range(S)]
        f = (rng.rand(D, 1) * 0.1 + 0.02)
        mu, var = np.zeros((D, 1)), np.ones((D, 1))
        amp = np.ones((D, 1)) * 0.5
        np.random.seed(9999)
        with tempfile.TemporaryDirectory() as tmp, contextlib.redirect_stdout(io.StringIO()):
            samples = du.generate_synthetic_data(tmp, cfg["N"], cfg["T"], cfg["label"], cfg["burn"], D, S, cfg["nlab"], 2,
                                                 A, nonlin, f, mu, var, amp, cfg["nl"], NOISE_TYPE=cfg["noise"])
        k = "gen%d" % c
        out[k + "/meta"] = json.dumps(cfg)
        out[k + "/A"], out[k + "/codes"], out[k + "/f"] = A, codes, f
        out[k + "/mu"], out[k + "/var"], out[k + "/amp"] = mu, var, amp
        out[k + "/X"] = np.stack([s[0] for s in samples])
        out[k + "/Y"] = np.stack([s[3] for s in samples])
        if c == 0:
            with tempfile.TemporaryDirectory() as tmp:
                with open(os.path.join(tmp, "subset_0.pkl"), "wb") as fh:
                    pickle.dump(samples, fh)
                with contextlib.redirect_stdout(io.StringIO()):
                    ds = sd.NormalizedSyntheticWVARDataset(tmp, shuffle=True, shuffle_seed=0, grid_search=False)
                    dsg = sd.NormalizedSyntheticWVARDataset(tmp, shuffle=True, shuffle_seed=0, grid_search=True)
                out["ds/means"] = np.asarray(ds.channel_means)
                out["ds/stds"] = ds.channel_std_devs.numpy()
                out["ds/order"] = np.array([j for _, j in ds.data])
                out["ds/order_gs"] = np.array([j for _, j in dsg.data])
                items = [ds[i] for i in range(3)]
                out["ds/x"] = np.stack([x.numpy() for x, _ in items])
                out["ds/y"] = np.stack([np.asarray(y) for _, y in items])
    np.savez_compressed(os.path.join(HERE, "svar_data.npz"), **out)
    print("wrote svar_data.npz (%d arrays)" % len(out))


if __name__ == "__main__":
    main()
