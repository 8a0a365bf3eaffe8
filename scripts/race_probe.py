#!/usr/bin/env python
"""Reproduce the round-1 intermittent A mismatch on demand (diagnostic, not a test).

k_emb_final's adjacency workgroup stages A, relu(A), the supports and dS into LDS (each thread
stores what it loaded), then forms the row sums of relu(A) -- entries stored by OTHER waves.
Round 1 had no barrier between the two, so a wave whose loads returned early could read rows a
later wave had not stored yet.  The variants built by redcliff_amd.build.build_variant delay
waves >= 1 before their staging pass (RC_PROBE_DELAY), which turns the rare timing into a
certain one:

  probe_fixed      delay + the barrier   -> A bit-identical to the production library
  probe_nobarrier  delay, no barrier     -> A differs in the rows / columns whose relu(A) rows
                                            waves >= 1 staged (p = 10: entries 64..99 = rows 6-9)

One D4IC-shaped pretrain-embedder step (which updates A through that workgroup) per library,
each in its own child process (the library is chosen by REDCLIFF_HIP_LIB before import).

    python scripts/race_probe.py            (parent: GPU work happens in the children)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd")
OUT = os.path.join(ROOT, "gpurun_out")


def child(tag):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import torch
    from test_gpu_replicas import data, make, opts
    m = make(0, 10.0, 0.1)
    oA, oB = opts(m, 5e-4, 2e-4)
    Xb, Yb = data(64, seed=7)[0]
    m.batch_update(0, 0, Xb, Yb, oA, oB, 1)  # pretrain-embedder step: Adam on A in k_emb_final
    torch.cuda.synchronize()
    A = m.factor_score_embedder.dgcnn.dgcnn.A.detach().cpu().numpy()
    np.save(os.path.join(OUT, "race_probe_%s.npy" % tag), A)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    sys.path.insert(0, PKG)
    from redcliff_amd import build as b
    import numpy as np
    os.makedirs(OUT, exist_ok=True)
    libs = {"production": b.LIB}
    libs.update((v, b.variant_path(v)) for v in b.VARIANTS)
    for tag, path in libs.items():
        if not os.path.exists(path):
            sys.exit("missing %s (build it on the CPU side: python -m redcliff_amd.build --variants)" % path)
        env = dict(os.environ, REDCLIFF_HIP_LIB=path, REDCLIFF_FORK="0")
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", tag], env=env, timeout=300)
        if r.returncode != 0:
            sys.exit("child %s failed with %d" % (tag, r.returncode))
    A = dict((t, np.load(os.path.join(OUT, "race_probe_%s.npy" % t))) for t in libs)
    rep = {}
    for t in libs:
        diff = A[t] != A["production"]
        rows = sorted(set(int(i) for i in np.nonzero(diff)[0]))
        cols = sorted(set(int(j) for j in np.nonzero(diff)[1]))
        rep[t] = {"entries_differing": int(diff.sum()), "of": int(diff.size), "rows": rows, "cols": cols,
                  "max_abs_diff": float(np.abs(A[t] - A["production"]).max())}
    print(json.dumps(rep, indent=1))
    ok = rep["probe_fixed"]["entries_differing"] == 0 and rep["probe_nobarrier"]["entries_differing"] > 0
    print("race reproduced without the barrier and absent with it" if ok else "UNEXPECTED probe outcome")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
