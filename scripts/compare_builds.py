"""Bitwise comparison of two library builds on the same fits (regression check for kernel
changes that must not change any bit).

    REDCLIFF_HIP_LIB=exp/lib_prev.so python scripts/compare_builds.py dump gpurun_out/prev.npz
    python scripts/compare_builds.py dump gpurun_out/cur.npz
    python scripts/compare_builds.py compare gpurun_out/prev.npz gpurun_out/cur.npz

dump: D4IC- and C1(K=4)-shaped fits (vector factor path) through pretrain -> acclimate ->
combined with a ragged last batch; every state_dict tensor is saved."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))


def dump(path):
    import bench
    import redcliff_amd
    out = {}
    for cfg in ("d4ic", "c1k4", "c4"):
        c = dict(bench.CONFIGS[cfg])
        m = bench.build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=0).cuda()
        oA, oB = bench.adam_pair(m, c)
        X, Y = bench.synth(c, 2 * c["B"] + 40, seed=3)
        bs = [(X[i:i + c["B"]], Y[i:i + c["B"]]) for i in range(0, X.shape[0], c["B"])]
        epochs = [int(e) for e in os.environ.get("COMPARE_EPOCHS", "0,1,2,3").split(",")]
        if os.environ.get("COMPARE_ONE_BATCH"):
            bs = bs[:1]
        if os.environ.get("COMPARE_BATCHES"):
            bs = bs[:int(os.environ["COMPARE_BATCHES"])]
        for epoch in epochs:
            for bi, (Xb, Yb) in enumerate(bs):
                m.batch_update(epoch, bi, Xb, Yb, oA, oB, 1)
        torch.cuda.synchronize()
        for k, v in m.state_dict().items():
            if not k.startswith("gen_model."):
                out["%s/%s" % (cfg, k)] = v.detach().cpu().numpy()
        for g, o in (("A", oA), ("B", oB)):
            for i, st in o.state_dict()["state"].items():
                for kk in ("exp_avg", "exp_avg_sq"):
                    if kk in st:
                        out["%s/opt%s/%d/%s" % (cfg, g, i, kk)] = st[kk].detach().cpu().numpy()
    np.savez(path, **out)
    print("dumped %d tensors to %s" % (len(out), path))


def compare(a, b):
    A, B = np.load(a), np.load(b)
    assert set(A.files) == set(B.files)
    bad = [k for k in A.files if not np.array_equal(A[k], B[k])]
    nshow = int(os.environ.get("COMPARE_SHOW", "20"))
    for k in bad[:nshow]:
        d = np.abs(A[k].astype(np.float64) - B[k])
        i = np.unravel_index(int(np.argmax(d)), d.shape) if d.ndim else ()
        rel = d / np.maximum(np.abs(A[k].astype(np.float64)), 1e-30)
        print("DIFF %s %s: max |d| %.3e at %s (a=%.6g b=%.6g), %d/%d differ, %d with rel > 1e-4"
              % (k, A[k].shape, float(d.max()), i, float(A[k][i]), float(B[k][i]), int((d > 0).sum()), d.size,
                 int((rel > 1e-4).sum())))
    print("%d / %d tensors differ" % (len(bad), len(A.files)))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        compare(sys.argv[2], sys.argv[3])
