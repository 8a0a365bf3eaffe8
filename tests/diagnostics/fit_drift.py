"""Per-epoch drift of a GPU fit from a reference fit fixture (tests/golden/<name>.npz).

    python tests/diagnostics/fit_drift.py <fixture name>

Runs the fit exactly as tests/test_gpu_fit_golden.py does (same model, windows and optimizers) under
whatever REDCLIFF_* environment the caller sets (kernel path / fc1 slice width), and prints, per
epoch, the relative deviation of the validation forecasting loss from the reference's, then the
largest relative deviation of the final state.  Used to tell rounding-order drift (changes with the
kernel path) from a systematic difference (the same whatever the path)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))
import test_gpu_fit_golden as T  # noqa: E402


def main(name):
    d, meta = T.load(name)
    m = T.build(meta)
    train, val = T.data(d, meta)
    oA, oB = T.opts(m, meta)
    m.fit(None, train, oA, oB, meta["L"], 1, 1, meta["max_iter"], val, **T.fit_kw(meta, d))
    h = m.fit_history
    got = np.asarray(h["avg_forecasting_loss"], np.float64)
    want = d["hist/avg_forecasting_loss"]
    n = min(len(got), len(want))
    env = " ".join("%s=%s" % (k, v) for k, v in sorted(os.environ.items()) if k.startswith("REDCLIFF_"))
    print("[%s] forecasting loss, signed rel dev per epoch: %s" % (env or "default", " ".join(
        "%+.2e" % ((got[i] - want[i]) / want[i]) for i in range(n))))
    fin = T.state(d, "final")
    worst = 0.0
    for k, v in m.state_dict().items():
        if k.startswith("gen_model.") or k.endswith("num_batches_tracked") or k not in fin:
            continue
        w = fin[k].astype(np.float64)
        g = v.detach().cpu().numpy().astype(np.float64)
        worst = max(worst, float(np.max(np.abs(g - w) / (np.abs(w) + 1e-3 * max(1.0, np.abs(w).max())))))
    print("[%s] final state: largest relative deviation %.2e" % (env or "default", worst))


if __name__ == "__main__":
    torch.cuda.set_device(0)
    main(sys.argv[1] if len(sys.argv) > 1 else "fit_tst_lag64")
