"""Bitwise comparison of two library builds on a packed fit's whole record: every history the
fit keeps (losses, GC-progress metrics, cosine similarities, confusion rates), best epochs and the
final parameters -- the check for kernel changes on the evaluation side (GC norms, GC-progress
statistics, validation values) that must not change any bit.

    [COMPARE_FITS_R=8] REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python scripts/compare_fits.py dump gpurun_out/fprev.npz
    python scripts/compare_fits.py dump gpurun_out/fcur.npz
    python scripts/compare_fits.py compare gpurun_out/fprev.npz gpurun_out/fcur.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))


def _flatten(prefix, obj, out):
    if isinstance(obj, dict):
        for k in sorted(obj, key=str):
            _flatten("%s/%s" % (prefix, k), obj[k], out)
    elif isinstance(obj, (list, tuple)) and obj and not np.isscalar(obj[0]) and not isinstance(obj[0], np.ndarray):
        for i, v in enumerate(obj):
            _flatten("%s/%d" % (prefix, i), v, out)
    elif isinstance(obj, (list, tuple)):
        out[prefix] = np.asarray([np.asarray(v, dtype=np.float64) for v in obj], dtype=np.float64)
    elif obj is None:
        return
    else:
        out[prefix] = np.asarray(obj, dtype=np.float64)


def dump(path):
    import torch
    import bench
    import redcliff_amd
    out = {}
    # COMPARE_FITS_CFGS=d4ic,c1k4,c4: the configurations (c4: K = 9, p = 12)
    for cfg in os.environ.get("COMPARE_FITS_CFGS", "d4ic,c1k4").split(","):
        c = dict(bench.CONFIGS[cfg])
        # COMPARE_FITS_R=8 or more: the packed (short-contraction matrix-core) factor kernels
        R, E = int(os.environ.get("COMPARE_FITS_R", "4")), 9
        models, opts = [], []
        for i in range(R):
            m = bench.build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=50 + i, pre=2, acc=1,
                                  forecast=(10.0, 1.0)[i % 2]).cuda()
            models.append(m)
            opts.append(bench.adam_pair(m, c))
        X, Y = bench.synth(c, 5 * c["B"], seed=11)
        B = c["B"]
        train = [(X[i:i + B], Y[i:i + B]) for i in range(0, 3 * B, B)]
        val = [(X[i:i + B], Y[i:i + B]) for i in range(3 * B, 5 * B, B)]
        rng = np.random.RandomState(7)
        true_gc = [(rng.rand(c["p"], c["p"], c["L"]) < 0.2).astype(np.float64) for _ in range(c["K"])]
        pack = redcliff_amd.ReplicaPack(models, opts)
        finals = pack.fit(None, train, val, max_iter=E, lookback=2, check_every=1, GC=true_gc)
        torch.cuda.synchronize()
        out["%s/finals" % cfg] = np.asarray(finals, dtype=np.float64)
        for r, m in enumerate(models):
            _flatten("%s/%d/hist" % (cfg, r), m.fit_history, out)
            for k, v in m.state_dict().items():
                out["%s/%d/state/%s" % (cfg, r, k)] = v.detach().cpu().numpy()
    np.savez(path, **out)
    print("dumped %d arrays to %s" % (len(out), path))


def compare(a, b):
    A, Bd = np.load(a), np.load(b)
    keys = sorted(set(A.files) | set(Bd.files))
    bad = []
    for k in keys:
        if k not in A.files or k not in Bd.files:
            bad.append((k, "missing"))
            continue
        x, y = A[k], Bd[k]
        if x.shape != y.shape or not np.array_equal(x, y, equal_nan=True):
            d = float(np.nanmax(np.abs(x - y))) if x.shape == y.shape else float("nan")
            bad.append((k, "max |diff| %.3g" % d))
    for k, why in bad[:40]:
        print("DIFF", k, why)
    print("%d / %d arrays differ" % (len(bad), len(keys)))
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
