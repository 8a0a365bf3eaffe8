"""ctypes binding of libredcliff_hip.so (include/redcliff_hip.h).

The library is the only compute path of this package on the GPU: there is no CPU or
eager-PyTorch fallback.  ``lib()`` raises ImportError when the shared object is missing
or does not export the expected ABI, so a broken build fails loudly.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB_PATH = os.path.join(_HERE, "lib", "libredcliff_hip.so")
LIB_PATH = os.environ.get("REDCLIFF_HIP_LIB", DEFAULT_LIB_PATH)
ABI_VERSION = 9

# RC_* step flags (include/redcliff_hip.h)
BN_TRAIN = 1 << 0
LOSS_FORECAST = 1 << 1
LOSS_FACTOR = 1 << 2
LOSS_FWL1 = 1 << 3
LOSS_ADJ = 1 << 4
STEP_A = 1 << 5
STEP_B = 1 << 6
VALUES = 1 << 7
CONFUSION = 1 << 8
STORE_OUTPUTS = 1 << 9
REFRESH_SUPPORTS = 1 << 10
GRAD_ONLY = 1 << 11

WS_REGIONS = ("T", "R", "f1", "w", "a", "y", "G", "G0", "w1", "gq", "ebp", "ecnt", "gfc1", "dwp", "dAadj", "dWi", "dS", "dgb", "S", "dZ", "amat",
              "lossp", "xsim", "gfc", "xw", "dyl", "dgs", "errw", "total")

EXPORTED = ("redcliff_abi_version", "redcliff_last_error", "redcliff_workspace_bytes", "redcliff_emb_param_count",
            "redcliff_fac_param_count", "redcliff_bn_batch_stats", "redcliff_dgcnn_supports", "redcliff_train_step",
            "redcliff_train_steps", "redcliff_workspace_layout", "redcliff_factor_forward",
            "redcliff_factor_forward_workspace_floats", "redcliff_step_predictions", "redcliff_gc_norms",
            "redcliff_prox", "redcliff_kernel_timing", "redcliff_kernel_times", "redcliff_adam_apply", "redcliff_dp_update", "redcliff_gemm",
            "redcliff_gc_progress", "redcliff_gc_progress_grouped", "redcliff_debug_guard_bands", "redcliff_workspace_regions",
            "redcliff_gc_track_stats", "redcliff_device_status", "redcliff_build_id")
KERNEL_IDS = ("supports", "emb_fwd", "fac_fwd", "fac_bwd", "emb_bwd", "emb_final", "fac_mix", "emb_combine", "fac_lead")


class Dims(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("R", "Bmax", "T", "p", "L", "K", "h", "F", "n", "H", "M1", "nsup",
                                               "use_sigmoid")] + [("sigmoid_ecc", ctypes.c_float)]


class AdamHyper(ctypes.Structure):
    _fields_ = [("lr", ctypes.c_double), ("beta1", ctypes.c_double), ("beta2", ctypes.c_double),
                ("eps", ctypes.c_float), ("weight_decay", ctypes.c_float), ("beta2_f", ctypes.c_float),
                ("one_minus_beta1_f", ctypes.c_float), ("one_minus_beta2_f", ctypes.c_float), ("t_offset", ctypes.c_int32)]


class ReplicaHyper(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in ("c_forecast", "c_factor", "c_cos", "c_fwl1", "c_smooth", "c_adj")] + [
        ("bn_eps", ctypes.c_double), ("bn_momentum", ctypes.c_double), ("A", AdamHyper), ("B", AdamHyper)]


_vp = ctypes.c_void_p
_i64 = ctypes.c_int64


class StepArgs(ctypes.Structure):
    _fields_ = [("d", Dims), ("B", ctypes.c_int32), ("flags", ctypes.c_int32), ("n_bn_updates", ctypes.c_int32),
                ("tA", ctypes.c_int32), ("tB", ctypes.c_int32),
                ("X", _vp), ("x_rstride", _i64), ("row0", _i64),
                ("labels", _vp), ("lab_rstride", _i64),
                ("bn_stats", _vp), ("bn_stats_rstride", _i64),
                ("emb", _vp), ("emb_m", _vp), ("emb_v", _vp), ("emb_stride", _i64),
                ("fac", _vp), ("fac_m", _vp), ("fac_v", _vp), ("fac_stride", _i64),
                ("bn_rm", _vp), ("bn_rv", _vp),
                ("hyper", _vp),
                ("ws", _vp), ("ws_bytes", ctypes.c_size_t),
                ("acc", _vp), ("confusion", _vp),
                ("B_global", ctypes.c_int32), ("pad_", ctypes.c_int32), ("grad_emb", _vp), ("grad_fac", _vp),
                ("replicas", _vp), ("n_replicas", ctypes.c_int32), ("pad2_", ctypes.c_int32)]


def adam_hyper(lr, betas, eps, weight_decay):
    b1, b2 = float(betas[0]), float(betas[1])
    return AdamHyper(float(lr), b1, b2, float(eps), float(weight_decay), b2, 1.0 - b1, 1.0 - b2, 0)


_LIB = None


def lib():
    """Load (once) and return the HIP library; raise ImportError if unavailable."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise ImportError("libredcliff_hip.so not built (%s); run __graft_entry__.build()" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    for name in EXPORTED:
        if not hasattr(L, name):
            raise ImportError("libredcliff_hip.so does not export %s" % name)
    L.redcliff_abi_version.restype = ctypes.c_int
    L.redcliff_last_error.restype = ctypes.c_char_p
    L.redcliff_workspace_bytes.restype = ctypes.c_size_t
    L.redcliff_workspace_bytes.argtypes = [ctypes.POINTER(Dims)]
    L.redcliff_emb_param_count.restype = ctypes.c_size_t
    L.redcliff_emb_param_count.argtypes = [ctypes.POINTER(Dims)]
    L.redcliff_fac_param_count.restype = ctypes.c_size_t
    L.redcliff_fac_param_count.argtypes = [ctypes.POINTER(Dims)]
    L.redcliff_bn_batch_stats.argtypes = [ctypes.POINTER(Dims), _vp, _i64, _i64, ctypes.c_int32, _vp, _i64, _vp]
    L.redcliff_dgcnn_supports.argtypes = [ctypes.POINTER(Dims), _vp, _i64, _vp, _vp]
    L.redcliff_train_step.argtypes = [ctypes.POINTER(StepArgs), _vp]
    L.redcliff_train_steps.argtypes = [ctypes.POINTER(StepArgs), ctypes.c_int32, _vp, _vp, ctypes.c_int32, _vp]
    L.redcliff_workspace_layout.argtypes = [ctypes.POINTER(Dims), ctypes.POINTER(_i64), ctypes.c_int32]
    L.redcliff_factor_forward.argtypes = [ctypes.POINTER(Dims), ctypes.c_int32, _vp, _i64, _vp, _i64, _vp, _i64, _vp,
                                          _i64, _vp]
    L.redcliff_factor_forward_workspace_floats.restype = ctypes.c_size_t
    L.redcliff_factor_forward_workspace_floats.argtypes = [ctypes.POINTER(Dims), ctypes.c_int32]
    L.redcliff_step_predictions.argtypes = [ctypes.POINTER(Dims), ctypes.c_int32, _vp, _vp, _i64, _vp]
    L.redcliff_gc_norms.argtypes = [ctypes.POINTER(Dims), _vp, _i64, _vp, _vp, _vp]
    L.redcliff_prox.argtypes = [ctypes.POINTER(Dims), _vp, _i64, ctypes.c_float, ctypes.c_float, ctypes.c_int32, _vp]
    L.redcliff_kernel_timing.argtypes = [ctypes.c_int32]
    L.redcliff_kernel_times.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_i64), ctypes.c_int32]
    L.redcliff_adam_apply.argtypes = [ctypes.POINTER(Dims), _vp, _vp, _vp, _vp, _i64, _i64, _vp, ctypes.c_int32,
                                      ctypes.c_int32, _vp]
    L.redcliff_dp_update.argtypes = [ctypes.POINTER(StepArgs), _i64, _i64, _vp]
    L.redcliff_gemm.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                ctypes.c_float, _vp, _i64, _i64, _vp, _i64, _i64, ctypes.c_float, _vp, _i64, _i64,
                                ctypes.c_int32, _vp]
    L.redcliff_gc_progress.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                       _vp, _vp, _vp, ctypes.c_double, ctypes.c_double, _vp, _vp]
    L.redcliff_gc_progress_grouped.argtypes = [ctypes.c_int32] * 6 + [_vp, _vp, _vp, ctypes.c_double, ctypes.c_double,
                                                                      _vp, _vp]
    L.redcliff_gc_track_stats.argtypes = [ctypes.c_int32, _i64, _vp, _vp, ctypes.c_int32, ctypes.c_int32, _i64, _vp,
                                          _vp, _vp]
    L.redcliff_debug_guard_bands.argtypes = [ctypes.c_int32]
    L.redcliff_device_status.argtypes = [ctypes.POINTER(Dims), _vp, ctypes.POINTER(ctypes.c_uint32), _vp]
    L.redcliff_workspace_regions.argtypes = [ctypes.POINTER(Dims), ctypes.POINTER(_i64), ctypes.c_int32]
    for name in EXPORTED[2:]:
        if name not in ("redcliff_workspace_bytes", "redcliff_emb_param_count", "redcliff_fac_param_count",
                        "redcliff_build_id"):
            getattr(L, name).restype = ctypes.c_int
    L.redcliff_build_id.restype = ctypes.c_char_p
    if L.redcliff_abi_version() != ABI_VERSION:
        raise ImportError("libredcliff_hip.so ABI %d != %d" % (L.redcliff_abi_version(), ABI_VERSION))
    want = tree_build_id()
    got = L.redcliff_build_id().decode()
    if want is not None and got != want:
        raise ImportError("libredcliff_hip.so was built from other sources (build id %s, this tree %s); run "
                          "__graft_entry__.build()" % (got, want))
    _LIB = L
    return L


def tree_build_id():
    """source_hash of the kernel sources next to this package, when the default in-tree library is
    the one loaded (REDCLIFF_HIP_LIB experiment builds and the trace / diagnostic variants carry
    their own defines and are not checked);
    None when the sources are not present."""
    if os.environ.get("REDCLIFF_HIP_LIB") or os.path.abspath(LIB_PATH) != os.path.abspath(DEFAULT_LIB_PATH):
        return None
    from . import build as _b
    if not _b.sources():
        return None
    return _b.source_hash()


def build_id():
    """The source hash compiled into the loaded library (redcliff_build_id)."""
    return lib().redcliff_build_id().decode()


def check(rc, what=""):
    if rc != 0:
        msg = lib().redcliff_last_error().decode(errors="replace")
        raise RuntimeError("redcliff HIP call %s failed (%d): %s" % (what, rc, msg))


def workspace_layout(dims):
    out = (_i64 * len(WS_REGIONS))()
    n = lib().redcliff_workspace_layout(ctypes.byref(dims), out, len(WS_REGIONS))
    if n < 0:
        check(n, "workspace_layout")
    return dict(zip(WS_REGIONS, [int(v) for v in out]))


def status_view(ws, ws_off, R):
    """int32 device view [R] of the replica status words of a workspace (WsOff.errw)."""
    return ws.as_strided((R,), (ws_off["total"],), ws_off["errw"]).view(torch.int32)


def raise_on_status(words, view=None, where="step"):
    """words: host copy of status_view (or redcliff_device_status's output).  Non-zero = a merged
    backward consumer stopped waiting for its producers (rc_wait_count ran out of polls), so the
    steps since the last check computed gradients from unwritten records: clear and raise."""
    import numpy as np
    w = np.asarray(words).reshape(-1)
    bad = np.nonzero(w)[0]
    if bad.size:
        if view is not None:
            view.zero_()
        raise RuntimeError("redcliff device status (%s): %d merged-backward hand-off wait(s) timed out in replica(s) %s "
                           "-- the affected training steps used unwritten gradient records; results are invalid "
                           "(set REDCLIFF_MERGE=0 to run the two-launch backward)" % (where, int(w[bad].sum()),
                                                                                     bad.tolist()))


def device_status(dims, ws, stream):
    """redcliff_device_status: read and clear the R status words (synchronises `stream`)."""
    out = (ctypes.c_uint32 * int(dims.R))()
    rc = lib().redcliff_device_status(ctypes.byref(dims), ws, out, stream)
    if rc < 0:
        check(rc, "device_status")
    return [int(v) for v in out]


def workspace_regions(dims):
    """[(start, size)] in floats of one replica's workspace regions (layout order)."""
    out = (_i64 * 80)()
    n = lib().redcliff_workspace_regions(ctypes.byref(dims), out, 40)
    if n < 0:
        check(n, "workspace_regions")
    return [(int(out[2 * i]), int(out[2 * i + 1])) for i in range(n)]


def guard_bands(floats):
    """Verification mode: guard bands of `floats` floats after every workspace region laid out
    from now on (0 = production layout).  Returns the previous setting."""
    return int(lib().redcliff_debug_guard_bands(int(floats)))


def kernel_timing(enable):
    lib().redcliff_kernel_timing(1 if enable else 0)


def kernel_times():
    """{kernel: (total_ms, launches)} for the launches recorded since the last call."""
    n = len(KERNEL_IDS)
    ms = (ctypes.c_double * n)()
    cnt = (_i64 * n)()
    rc = lib().redcliff_kernel_times(ms, cnt, n)
    if rc < 0 or rc > 1000:
        check(rc, "kernel_times")
    return dict((k, (float(ms[i]), int(cnt[i]))) for i, k in enumerate(KERNEL_IDS))
