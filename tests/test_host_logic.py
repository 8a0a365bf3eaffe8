"""CPU tests of the host-side mirror: parameter trees / seeded init against the reference's
golden vectors, the phase schedule, label selection, and loud failure without a GPU."""
import numpy as np
import pytest
import torch

from golden_io import SCENARIOS, ctor_args, load, state
from oracle.redcliff_oracle import OracleREDCLIFF


def build(meta):
    import redcliff_amd
    args, kw = ctor_args(meta)
    torch.manual_seed(meta["seed"])
    cls = redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing if meta["smoothing_class"] else redcliff_amd.REDCLIFF_S_CMLP
    return cls(*args, **kw).float()


@pytest.mark.parametrize("name", [s for s in SCENARIOS])
def test_seeded_init_matches_reference(name):
    d, meta = load(name)
    m = build(meta)
    want = state(d, "init")
    got = dict((k, v) for k, v in m.state_dict().items() if not k.startswith("gen_model."))
    assert set(got) == set(want)
    for k in want:
        np.testing.assert_array_equal(got[k].numpy(), want[k], err_msg=k)


def test_phase_schedule_matches_oracle():
    from redcliff_amd.engine import phase_of_epoch
    d, meta = load("dgcnn_c1")
    args, kw = ctor_args(meta)
    for mode, pre, acc in [("pretrain_embedder_then_acclimate_factors_then_combined", 2, 3),
                           ("pretrain_embedder_then_combined", 2, 0), ("combined", 0, 0),
                           ("pretrain_embedder_and_pretrain_factor_then_combined", 1, 0),
                           ("pretrain_embedder_then_post_train_factor", 2, 0)]:
        kw2 = dict(kw, training_mode=mode, num_pretrain_epochs=pre, num_acclimation_epochs=acc)
        torch.manual_seed(0)
        o = OracleREDCLIFF(*args, **kw2)
        torch.manual_seed(0)
        m = build(dict(meta, training_mode=mode, pre=pre, acc=acc))
        for ep in range(8):
            want = list(o.phase(ep))
            want = [w for w in want if w is not None]
            assert phase_of_epoch(m, ep) == want, (mode, ep)


def test_label_selection_rules():
    from redcliff_amd.engine import select_labels
    Y = torch.arange(2 * 3 * 10, dtype=torch.float32).view(2, 3, 10)
    assert torch.equal(select_labels(Y, 3, 5), Y[:, :, 5])        # T_y > Lmax: label at Lmax (:637)
    Y1 = Y[:, :, :1]
    assert torch.equal(select_labels(Y1, 3, 5), Y1[:, :, 0])      # D4IC: (N, K, 1)
    Y2 = Y[:, :, 0]
    assert torch.equal(select_labels(Y2, 3, 5), Y2)               # 2-D labels
    assert select_labels(Y2[:, :2], 3, 5).shape == (2, 3)          # fewer label columns than factors


def test_compute_without_gpu_fails_loudly():
    d, meta = load("dgcnn_c1")
    m = build(meta)
    X = torch.from_numpy(d["X"][:4])
    with pytest.raises(RuntimeError, match="GPU"):
        m(X[:, :5])


def test_step_flags_after_prior_factors():
    """A model whose factors came from prior_factors_path keeps training its embedder but never
    steps optimizerB again (the reference's optimizerB keeps the replaced parameters); updates
    that would only move the factors change nothing and are skipped."""
    from redcliff_amd import _native as nat
    from redcliff_amd.engine import flags_for, step_flags
    d, meta = load("dgcnn_c1")
    m = build(meta)
    for kind in ("pretrain_embedder", "pretrain_factor", "acclimate", "post_train", "combined"):
        assert step_flags(m, kind, 2) == flags_for(kind, 2)
    m.__dict__["_factors_detached"] = True
    for kind in ("pretrain_factor", "acclimate", "post_train"):
        assert step_flags(m, kind, 2) == (0, 0)
    for kind in ("pretrain_embedder", "combined"):
        f, nbn = step_flags(m, kind, 2)
        f0, nbn0 = flags_for(kind, 2)
        assert f == f0 & ~nat.STEP_B and f & nat.STEP_A and nbn == nbn0


def test_freeze_decision_raises_like_the_reference():
    """determine_which_factors_need_updates on the (p, p, 1) lag-free estimates: numpy's
    norm(ord=1) of a 3-d array raises, exactly as in the reference (...withStateSmoothing.py:
    1159-1166)."""
    x = np.random.RandomState(0).rand(5, 5, 1).astype(np.float32)
    with pytest.raises(ValueError, match="Improper number of dimensions to norm"):
        np.linalg.norm(x / np.max(x), ord=1)


def test_packed_fit_module_modes_match_torch_eval():
    """replicas._eval_modes (the flags a packed fit leaves, written through the module dicts listed
    when the pack is built) sets exactly the flags torch's recursive .eval() on the embedder and
    every factor sets (...withStateSmoothing.py:1366-1480), and leaves the other modules alone."""
    import copy
    import bench
    import redcliff_amd
    from redcliff_amd import replicas
    c = bench.CONFIGS["d4ic"]
    ms = [bench.build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=s) for s in range(3)]
    ref = copy.deepcopy(ms)
    for m in ref:
        m.factor_score_embedder.eval()
        for f in m.factors:
            f.eval()
    replicas._eval_modes(ms[:1])                              # walking the trees
    replicas._eval_modes(ms[1:], replicas._module_dicts(ms[1:]))  # the pack's precomputed list
    for a, b in zip(ms, ref):
        flags_a = [(n, x.training) for n, x in a.named_modules()]
        flags_b = [(n, x.training) for n, x in b.named_modules()]
        assert flags_a == flags_b
    assert any(t for _, t in flags_a)  # modules outside the embedder / factors keep their mode
