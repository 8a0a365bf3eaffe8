"""Per-kernel workgroup timing of the fused step (trace build, -DRC_TRACE).

    python scripts/phase_trace.py [--config d4ic]

Loads libredcliff_hip_trace.so, runs a few combined-phase steps of bench.py's workload and
prints, for the last step, each kernel's start (relative to the first), span, start spread
of its workgroups and their duration distribution (RC_WG_MARK slots, 100 MHz wall clock).
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
    # REDCLIFF_TRACE_LIB: a prebuilt trace variant (scripts/build_tree.sh <name> -DRC_TRACE ...)
    _native.LIB_PATH = os.environ.get("REDCLIFF_TRACE_LIB") or b.build(trace=True)
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
    tr = eng.ws[tot - 32768:tot].cpu().numpy().view(np.uint64).astype(np.int64).reshape(8, 2048)
    names = ["emb_fwd", "fac_fwd", "fac_bwd", "emb_bwd", "emb_final", "fac_mix"]
    # merged backward: node workgroups' wait-return times (kid 7, start slots only)
    wt = tr[7][0::2]
    wt = wt[wt > 0]
    t_first = min(int(tr[k][0::2][tr[k][0::2] > 0].min()) for k in range(len(names)) if (tr[k][0::2] > 0).any())
    ph = tr[6]
    for lo, hi, label in ((0, 16, "emb_fwd WG0 phases"), (16, 32, "fac_bwd WG0 phases"), (32, 48, "emb_bwd WG0 phases"),
                            (48, 64, "emb_final adjacency WG phases")):
        t = ph[lo:hi]
        idx = [i for i in range(hi - lo) if t[i] > 0]
        if len(idx) > 1:
            print(label + ": " + "  ".join("%d->%d %.2f" % (lo + a, lo + b, (t[b] - t[a]) / 100.0) for a, b in zip(idx, idx[1:])))
    if ph[32] > 0:  # the embedder backward's node workgroup 0 marks in slot order, us after mark 32
        print("emb_bwd WG0 marks (us after 32): " +
              "  ".join("%d %.2f" % (i, (ph[i] - ph[32]) / 100.0) for i in range(32, 48) if ph[i] > 0))
    if ph[48] > 0:  # the adjacency workgroup's marks in slot order, us after mark 48
        print("emb_final adjacency WG marks (us after 48): " +
              "  ".join("%d %.2f" % (i, (ph[i] - ph[48]) / 100.0) for i in range(48, 64) if ph[i] > 0))
    upd = [(i, (ph[i] - t_first) / 100.0) for i in range(19, 24) if ph[i] > 0]
    if upd:  # the (network 0, chunk 1) factor workgroup's update part (rc_fac_bwd.h, trace builds)
        print("factor update WG (network 0, chunk 1) phases at: " + "  ".join("%d %.2f us" % x for x in upd))
    for k, name in enumerate(names):
        st, en = tr[k][0::2], tr[k][1::2]
        ok = (st > 0) & (en > 0)
        if not ok.any():
            continue
        st, en = st[ok], en[ok]
        dur = (en - st) / 100.0
        print("%-9s WGs %4d  start %7.2f us  span %7.2f us  start spread %6.2f  WG dur min/med/max %6.2f %6.2f %6.2f"
              % (name, ok.sum(), (st.min() - t_first) / 100.0, (en.max() - st.min()) / 100.0,
                 (st.max() - st.min()) / 100.0, dur.min(), np.median(dur), dur.max()))


    pub = tr[7][1::2]
    pub = pub[pub > 0]
    if pub.size:
        print("factor leads published (merged backward): %d leads, first %.2f us  median %.2f  last %.2f"
              % (pub.size, (pub.min() - t_first) / 100.0, (np.median(pub) - t_first) / 100.0,
                 (pub.max() - t_first) / 100.0))
        order = np.argsort(tr[7][1::2])[::-1][:5]
        print("  latest leads (workgroup: publish us): %s" % ", ".join(
            "%d: %.2f" % (i, (tr[7][1::2][i] - t_first) / 100.0) for i in order if tr[7][1::2][i] > 0))
    if wt.size:
        print("emb wait returned (merged backward node WGs): %d WGs, first %.2f us  median %.2f  last %.2f"
              % (wt.size, (wt.min() - t_first) / 100.0, (np.median(wt) - t_first) / 100.0, (wt.max() - t_first) / 100.0))


if __name__ == "__main__":
    main()
