"""CPU-side checks of the C-ABI library: it loads, exports every entry point that
include/redcliff_hip.h declares, and its host-only helpers agree with the Python layout.
No kernel is launched here."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "redcliff_hip.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|size_t|const char\*)\s+(redcliff_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_declared_symbol():
    from redcliff_amd import _native as nat
    L = nat.lib()
    syms = declared_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(L, s), s
        assert s in nat.EXPORTED, "binding does not cover " + s
    assert L.redcliff_abi_version() == nat.ABI_VERSION


def c1_dims(Bmax=128, T=100):
    from redcliff_amd import _native as nat
    return nat.Dims(R=1, Bmax=Bmax, T=T, p=10, L=5, K=4, h=25, F=16, n=3, H=100, M1=64, nsup=4, use_sigmoid=0,
                    sigmoid_ecc=0.0)


def test_param_counts_match_python_layout():
    from redcliff_amd import _native as nat
    from redcliff_amd.kernels import factor_layout
    d = c1_dims()
    L = nat.lib()
    assert L.redcliff_fac_param_count(ctypes.byref(d)) == factor_layout(4, 10, 25, 5)["total"] == 52040
    # DGCNN(16, 10, 3, 100, 4): A 100 + gc 3*16*100 + bn 32 + fc1 64*1000+64 + fc2 4*64+4
    assert L.redcliff_emb_param_count(ctypes.byref(d)) == 100 + 4800 + 32 + 64064 + 260


def test_workspace_layout_and_validation():
    from redcliff_amd import _native as nat
    L = nat.lib()
    d = c1_dims()
    nbytes = L.redcliff_workspace_bytes(ctypes.byref(d))
    lay = nat.workspace_layout(d)
    assert nbytes == 4 * lay["total"]
    offs = [lay[k] for k in nat.WS_REGIONS]
    assert offs == sorted(offs) and all(o % 64 == 0 for o in offs)
    bad = c1_dims()
    bad.p = 65
    assert L.redcliff_workspace_bytes(ctypes.byref(bad)) == 0
    assert b"limits" in L.redcliff_last_error()
    bad = c1_dims()
    bad.F = 3  # embed_lag < gen_lag is outside the fused path
    assert L.redcliff_workspace_bytes(ctypes.byref(bad)) == 0


def test_guard_band_layout():
    """Verification layout (redcliff_debug_guard_bands): every region is followed by its own band,
    bands never overlap the next region, and the last band closes the replica's slice."""
    from redcliff_amd import _native as nat
    d = c1_dims()
    plain = nat.workspace_regions(d)
    assert len(plain) == 35 and nat.workspace_layout(d)["total"] >= plain[-1][0] + plain[-1][1]
    prev = nat.guard_bands(64)
    try:
        regs = nat.workspace_regions(d)
        total = nat.workspace_layout(d)["total"]
        assert [n for _, n in regs] == [n for _, n in plain]
        for (s, n), (s2, _) in zip(regs, regs[1:]):
            assert s % 64 == 0 and s + n + 64 <= s2
        assert regs[-1][0] + regs[-1][1] + 64 <= total
        assert nat.lib().redcliff_workspace_bytes(ctypes.byref(d)) == 4 * total
    finally:
        nat.guard_bands(prev)
    assert nat.workspace_regions(d) == plain


def test_train_step_rejects_null_arguments():
    from redcliff_amd import _native as nat
    L = nat.lib()
    a = nat.StepArgs()
    a.d = c1_dims()
    a.B = 16
    rc = L.redcliff_train_step(ctypes.byref(a), None)
    assert rc == -1 and b"null" in L.redcliff_last_error()


def test_build_id_matches_committed_sources():
    """The library carries the hash of the sources it was compiled from (redcliff_build_id), and
    build() treats a library as current only when that hash equals the tree's (not by mtime)."""
    from redcliff_amd import _native as nat
    from redcliff_amd import build as b
    want = b.source_hash()
    assert re.fullmatch(r"[0-9a-f]{16}", want)
    assert b.embedded_id(b.LIB) == want
    assert nat.build_id() == want
    assert not b._stale(b.LIB)
    # a define changes the id (experiment variants never pass for the product library)
    assert b.source_hash(["-DRC_TRACE"]) != want
