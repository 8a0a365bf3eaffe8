"""Per-phase wall-clock breakdown of the fused step (trace build, -DRC_TRACE).

    python scripts/phase_trace.py [--config d4ic]

Loads libredcliff_hip_trace.so, runs a few combined-phase steps of bench.py's workload and
prints the deltas between the RC_MARK slots (100 MHz wall clock) of the last step.
Slot map: 256+i = embedder-backward node workgroup 0 (i = 0..7); 600+2b / 601+2b = start / end of node block b.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd")
sys.path.insert(0, ROOT)
sys.path.insert(0, PKG)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="d4ic")
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    from redcliff_amd import build as b
    from redcliff_amd import _native
    assert _native._LIB is None
    _native.LIB_PATH = b.build(trace=True)
    import numpy as np
    import torch
    import bench
    import redcliff_amd
    c = bench.CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    model = bench.build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=0).to(dev)
    oA, oB = bench.adam_pair(model, c)
    X, Y = bench.synth(c, 4 * c["B"], seed=1)
    loader = [(X[i:i + c["B"]], Y[i:i + c["B"]]) for i in range(0, X.shape[0], c["B"])]
    eng = model.engine()
    ds = eng.cache_dataset(loader)
    d = eng.workspace(ds["Bmax"], ds["T"])
    idx = np.arange(args.steps) % len(loader)
    stats = ds["stats"][torch.as_tensor(idx, device=dev)].contiguous()
    eng.run_steps(["combined"], ds["X"], ds["lab"], stats, d, ds["rows"][idx], ds["sizes"][idx], oA, oB)
    torch.cuda.synchronize()
    tot = eng.ws_off["total"]
    tr = eng.ws[tot - 4096:tot].cpu().numpy().view(np.uint64).astype(np.int64)
    def span(lo, hi, label):
        t = tr[lo:hi]
        print("%s:" % label)
        for i in range(1, len(t)):
            if t[i] and t[i - 1]:
                print("  mark %d -> %d : %8.2f us" % (lo + i - 1, lo + i, (t[i] - t[i - 1]) / 100.0))
    span(256, 264, "emb_bwd node WG 0 (marks 5/6 only if it arrived last; 7 = ticket)")
    se = tr[600:2000].reshape(-1, 2)
    se = se[(se[:, 0] > 0) & (se[:, 1] > 0)]
    if len(se):
        t0 = se[:, 0].min()
        dur = (se[:, 1] - se[:, 0]) / 100.0
        print("emb_bwd node blocks: %d traced; start spread %.2f us; end max %.2f us after first start" % (
            len(se), (se[:, 0].max() - se[:, 0].min()) / 100.0, (se[:, 1].max() - t0) / 100.0))
        print("  duration min/median/max %.2f / %.2f / %.2f us" % (dur.min(), np.median(dur), dur.max()))



if __name__ == "__main__":
    main()
