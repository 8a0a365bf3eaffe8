"""Per-workgroup timing of replica 0's workgroups in a packed grid step (trace build, -DRC_TRACE).

    python scripts/phase_trace_pack.py [--replicas 128] [--config d4ic]

Loads libredcliff_hip_trace.so, runs bench.py's grid leg for a few steps and prints, for the last
step, each traced kernel's span over replica 0's workgroups and their duration distribution
(RC_WG_MARK slots; in k_emb_final workgroup 0 is the adjacency workgroup).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=128)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--config", default="d4ic")
    args = ap.parse_args()
    from redcliff_amd import build as b
    from redcliff_amd import _native
    _native.LIB_PATH = b.build(trace=True)
    import numpy as np
    import torch
    import bench
    import redcliff_amd
    packs = []
    orig = redcliff_amd.ReplicaPack.__init__

    def capture(self, *a, **k):
        orig(self, *a, **k)
        packs.append(self)
    redcliff_amd.ReplicaPack.__init__ = capture
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c = bench.CONFIGS[args.config]
    ns = argparse.Namespace(replicas=args.replicas, grid_steps=args.steps)
    el, R, steps = bench.run_grid(c, ns, dev, 0, None)
    torch.cuda.synchronize()
    pack = packs[-1]
    tot = pack.ws_off["total"]
    tr = pack.ws[tot - 32768:tot].cpu().numpy().view(np.uint64).astype(np.int64).reshape(8, 2048)
    names = ["emb_fwd", "fac_fwd", "fac_bwd", "emb_bwd", "emb_final", "fac_mix"]  # RC_KID_* (packed grid: emb_fwd =
    # k_lemb_prep_win, emb_bwd = k_lemb_win_bwd, fac_fwd / fac_bwd = the s16 kernels)
    starts = [tr[k][0::2][tr[k][0::2] > 0] for k in range(len(names))]
    t_first = min(int(s.min()) for s in starts if s.size)
    for k, name in enumerate(names):
        st, en = tr[k][0::2], tr[k][1::2]
        ok = (st > 0) & (en > 0)
        if not ok.any():
            continue
        dur = (en[ok] - st[ok]) / 100.0
        print("%-9s WGs %4d  start %8.2f us  span %7.2f us  WG dur min/med/max %6.2f %6.2f %6.2f  WG0 %6.2f"
              % (name, ok.sum(), (st[ok].min() - t_first) / 100.0, (en[ok].max() - st[ok].min()) / 100.0,
                 dur.min(), np.median(dur), dur.max(), (en[0] - st[0]) / 100.0 if ok[0] else -1), flush=True)
    # phase marks of workgroup 0 of replica 0 (RC_PHASE slots 6 * 2048 + i), per kernel relative to
    # its first mark: k_lemb_win_bwd 0..7, k_lemb_prep_win 8..15, k_fac_mix 16..23, k_emb_final 48..58
    ph = tr[6]
    for name, lo, hi in (("lemb_win_bwd", 0, 8), ("lemb_prep_win", 8, 16), ("fac_mix", 16, 24), ("emb_final", 48, 64)):
        marks = [(i, int(ph[i])) for i in range(lo, hi) if ph[i] > 0]
        if marks:
            print("phase marks %-13s (us after its first mark): " % name +
                  " ".join("%d:%.2f" % (i, (t - marks[0][1]) / 100.0) for i, t in marks), flush=True)

if __name__ == "__main__":
    main()
