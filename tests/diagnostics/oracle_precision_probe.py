"""How well-conditioned a fit fixture's float32 training step is: the oracle (oracle/redcliff_oracle.py,
which reproduces the reference's fit fixtures bit for bit on the CPU) in float32 against the same
seeded model converted to float64, after the first training step(s), per embedder tensor.

    python tests/diagnostics/oracle_precision_probe.py <fixture name> [steps]

fit_tst_lag64 (flat-start windows: 60 of the 64 embedder time steps are a constant 0.00291 with a
4e-5 spread across windows) moves by up to 2.8e-3 of a tensor's scale between the two precisions after
ONE step, in exactly the tensors and magnitudes by which the GPU fit leaves the reference
(profiles/r06_step_drift_lag64.log); fit_tst stays below 1e-5.  CPU only (test infrastructure)."""
import copy
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle.redcliff_oracle import OracleREDCLIFF, make_optimizers  # noqa: E402


def main(name, steps):
    torch.set_num_threads(8)
    d = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
    meta = json.loads(str(d["meta"]))
    eargs = [("num_features_per_node", meta["F"]), ("num_graph_conv_layers", meta["n"]),
             ("num_hidden_nodes", meta["H"]), ("sigmoid_eccentricity_coeff", 10.0)]
    torch.manual_seed(meta["seed"])
    o32 = OracleREDCLIFF(meta["p"], meta["L"], [meta["h"]], meta["F"], [0], meta["L"], 1, meta["K"], meta["nsup"],
                         meta["coeff"], False, "DGCNN", eargs, "conditional_factor_fixed_embedder",
                         "apply_factor_weights_after_sim_completion", num_sims=1, wavelet_level=None, save_path=None,
                         training_mode="pretrain_embedder_then_acclimate_factors_then_combined",
                         num_pretrain_epochs=meta["pre"], num_acclimation_epochs=meta["acc"],
                         STATE_SCORE_SMOOTHING_EPSILON=0.0001)
    o64 = copy.deepcopy(o32).double()
    B = meta["B"]
    X, Y = [torch.from_numpy(d[k]) for k in ("X", "Y")]
    res = {}
    for tag, o, dt in (("f32", o32, torch.float32), ("f64", o64, torch.float64)):
        torch.set_default_dtype(dt)
        oA, oB = make_optimizers(o, meta["lrA"], 1e-4, 1e-4, meta["lrB"], 1e-4, 1e-4)
        for s in range(steps):
            bi = s % 2
            o.batch_update(s // 2, bi, X[bi * B:(bi + 1) * B].to(dt), Y[bi * B:(bi + 1) * B].to(dt), oA, oB, 1)
        res[tag] = dict((k, v.detach().double()) for k, v in o.state_dict().items() if not k.startswith("gen_model."))
    torch.set_default_dtype(torch.float32)
    rows = []
    for k in res["f32"]:
        if k.endswith("num_batches_tracked") or "factor_score_embedder" not in k:
            continue
        w, g = res["f64"][k], res["f32"][k]
        rows.append((float((g - w).abs().max()) / (float(w.abs().max()) or 1.0), k))
    rows.sort(reverse=True)
    print(name, "f32 vs f64 oracle:", "; ".join("%s %.2e" % (k.split("dgcnn.")[-1], e) for e, k in rows[:8]))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
