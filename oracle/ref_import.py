"""TEST INFRASTRUCTURE ONLY -- import the reference's Python hot path in THIS container.

Used solely by ``tests/golden/make_golden.py`` to generate golden vectors from the
reference itself.  ``/root/reference`` does not exist on the GPU box, so nothing that
runs there (``-m gpu`` tests, ``smoke()``, ``bench.py``) may import this module.

Two third-party imports of the reference are absent from the image:
* ``pywt`` (pywavelets 1.8.0, ``general_utils/time_series.py:2``) -- never called on the
  hot path (``wavelet_level=None``): an empty module stands in for the import;
* ``torcheeg`` (1.1.3, ``models/dgcnn.py:9``) -- its DGCNN is restated in
  ``oracle/torcheeg_dgcnn.py`` ("parity unpinned at the torcheeg 1.1.3 boundary").
"""
import os
import sys
import types

REF_ROOT = os.environ.get("REDCLIFF_REFERENCE_ROOT", "/root/reference")


def reference_available():
    return os.path.isdir(os.path.join(REF_ROOT, "models"))


def import_reference():
    """Return a namespace with the reference modules the hot path uses."""
    if not reference_available():
        raise RuntimeError("reference tree not present at %s" % REF_ROOT)
    import matplotlib
    matplotlib.use("Agg")
    if "pywt" not in sys.modules:
        sys.modules["pywt"] = types.ModuleType("pywt")
    if "torcheeg" not in sys.modules:
        from oracle import torcheeg_dgcnn
        pkg = types.ModuleType("torcheeg")
        mdl = types.ModuleType("torcheeg.models")
        mdl.DGCNN = torcheeg_dgcnn.DGCNN
        pkg.models = mdl
        sys.modules["torcheeg"] = pkg
        sys.modules["torcheeg.models"] = mdl
    if REF_ROOT not in sys.path:
        sys.path.insert(0, REF_ROOT)
    import importlib
    ns = types.SimpleNamespace()
    ns.cmlp = importlib.import_module("models.cmlp")
    ns.embedders = importlib.import_module("models.redcliff_factor_score_embedders")
    ns.redcliff = importlib.import_module("models.redcliff_s_cmlp")
    ns.redcliff_smooth = importlib.import_module("models.redcliff_s_cmlp_withStateSmoothing")
    ns.metrics = importlib.import_module("general_utils.metrics")
    ns.model_utils = importlib.import_module("general_utils.model_utils")
    return ns
