"""The reference's own fp32 spread around the fit fixtures (CPU; tests/golden/make_fit_envelope.py).

Each envelope holds realizations of the reference's ``fit`` (and of its fresh-optimizer resume) that
differ from the fixture only in the rounding order of torch's reductions over the window axis (the
rows of every training batch permuted; one CPU thread instead of eight).  These checks pin what
tests/test_gpu_fit_golden.py relies on when it bounds the GPU fit by that spread:
  * every realization takes the fixture's decisions (stopping epoch, best_it): the spread is
    rounding, not a different trajectory;
  * realization 0 (the fixture's own window order) stays within 1e-3 of the fixture along the fit;
  * fit_tst_lag64's envelope adds a float64 realization (ENVELOPE_DTYPE=float64, the fixture's window
    order): its flat-start windows make the float32 computation ill-conditioned, so the float64 run
    leaves the window-order spread by far while taking the same decisions;
  * the resumed C1 fit's spread exceeds the 1e-4 loss tolerance (measured 2.2e-3 on the last fw-L1
    entry) and its states leave the 2e-4 state tolerance at dozens of entries -- the reason the
    resume test cannot hold the fixed tolerance for any implementation, the reference included.
"""
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
HKEYS = ["avg_forecasting_loss", "avg_factor_loss", "avg_factor_cos_sim_penalty", "avg_fw_l1_penalty",
         "avg_fw_smoothing_penalty", "avg_adj_penalty", "avg_dagness_reg_loss", "avg_dagness_lag_loss",
         "avg_dagness_node_loss", "avg_combo_loss"]
SCENARIOS = [n for n in ("fit_c1", "fit_d4ic", "fit_d4ic_pub", "fit_tst", "fit_tst_lag64") if os.path.exists(os.path.join(GOLDEN, n + "_envelope.npz"))]


def _load(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    e = np.load(os.path.join(GOLDEN, name + "_envelope.npz"), allow_pickle=False)
    return d, e


def _spread(d, e, part, href):
    worst = 0.0
    for k in HKEYS:
        want = d["%s/%s" % (href, k)]
        rows = e["%s/hist/%s" % (part, k)]
        rel = np.abs(rows - want) / np.maximum(np.abs(want), 1e-6)
        worst = max(worst, float(np.nanmax(rel)) if rel.size else 0.0)
    return worst


@pytest.mark.parametrize("name", SCENARIOS)
def test_realizations_take_the_fixture_decisions(name):
    d, e = _load(name)
    assert int(e["J"]) >= 4
    for part, href in (("fit", "hist"), ("resume", "resume/hist")):
        np.testing.assert_array_equal(e[part + "/epoch"], int(d[href + "/epoch"]))
        np.testing.assert_array_equal(e[part + "/best_it"], int(d[href + "/best_it"]))
        for k in HKEYS:
            rows = e["%s/hist/%s" % (part, k)]
            assert rows.shape == (int(e["J"]),) + d["%s/%s" % (href, k)].shape, (part, k)
            assert not np.isnan(rows).any(), (part, k)
    # realization 0 (the fixture's window order, one thread): close to the fixture along the fit (the
    # resumed fit amplifies even the thread-count difference past 1e-3: C1's last fw-L1 entry)
    for k in HKEYS:
        np.testing.assert_allclose(e["fit/hist/%s" % k][0], d["hist/%s" % k], rtol=1e-3, atol=1e-6)


def test_resumed_c1_spread_exceeds_the_fixed_tolerance():
    if "fit_c1" not in SCENARIOS:
        pytest.skip("fit_c1 envelope not generated")
    d, e = _load("fit_c1")
    assert _spread(d, e, "fit", "hist") < 1e-4
    assert _spread(d, e, "resume", "resume/hist") > 1e-3
    outside = sum(e[k] for k in e.files if k.startswith("resume/outside/"))
    assert int(np.max(outside)) > 10
    meta = json.loads(str(d["meta"]))
    assert meta["lrA"] == meta["lrB"] == 5e-4
