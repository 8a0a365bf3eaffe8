"""Register budgets of the hot kernels, read from the built library's gfx950 code object (CPU only).

Several round-5 changes were bit-identical and faster where measured, but added live values to a
kernel already at a register boundary: the multi-sub-block embedder backward went from 256 to
256 + 32 registers (one wave per SIMD instead of two) and the data-parallel leg lost a quarter of
its speed.  Occupancy is a property of the compiled code, so it is checked
here, from the kernel descriptors' metadata (llvm-readelf --notes), not on the GPU.
"""
import glob
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd", "redcliff_amd", "lib", "libredcliff_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"

# kernel (substring of the mangled name) -> minimum waves per SIMD
MIN_WAVES = {
    "k_forwardILi1E": 4,          # single-fit forward (one window per workgroup)
    "k_emb_bwdILb0E": 3,          # single-sub-block embedder backward
    "k_emb_bwdILb1E": 2,          # multi-sub-block (data-parallel B = 512 shard steps)
    "k_bwd_mergedILb0E": 2,       # merged backward (the D4IC `value` step)
    "k_bwd_mergedILb1E": 2,
    "k_emb_tailILi4E": 2,
    "k_emb_finalILi4E": 2,
    "k_fac_bwdE": 2,
    "k_fac_bwd_s16ILi16E": 3,     # RC_S16_BWD_WAVES (the packed grid)
    "k_emb_combineE": 8,
}
# single-fit kernels that must not touch scratch
NO_SCRATCH = ["k_forwardILi1E", "k_emb_bwdILb0E", "k_emb_bwdILb1E", "k_bwd_mergedILb0E", "k_emb_tailILi4E",
              "k_emb_finalILi4E"]


def _kernels(tmp):
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    objdump, readelf = os.path.join(LLVM, "llvm-objdump"), os.path.join(LLVM, "llvm-readelf")
    if not (os.path.exists(objdump) and os.path.exists(readelf)):
        pytest.skip("llvm-objdump / llvm-readelf not in the image")
    lib = os.path.join(tmp, "lib.so")
    shutil.copy(LIB, lib)  # the bundles are extracted next to the input
    subprocess.run([objdump, "--offloading", lib], capture_output=True, check=True, cwd=tmp)
    out = {}
    for obj in glob.glob(lib + ".*gfx950"):
        notes = subprocess.run([readelf, "--notes", obj], capture_output=True, text=True, check=True).stdout
        for blk in re.split(r"\n\s+- \.agpr_count:", notes)[1:]:
            def field(k):
                m = re.search(r"\." + k + r":\s+(\S+)", blk)
                return m.group(1) if m else None
            name = field("name")
            if name and field("vgpr_count"):
                out[name] = {"vgpr": int(field("vgpr_count")), "scratch": int(field("private_segment_fixed_size") or 0)}
    if not out:
        pytest.skip("no gfx950 kernel metadata found")
    return out


def _waves(vgpr):
    # .vgpr_count is the unified (architectural + accumulation) count; 512 per SIMD lane, granule 8
    return min(8, 512 // (((vgpr + 7) // 8) * 8))


def test_hot_kernels_keep_their_waves_per_simd(tmp_path):
    ks = _kernels(str(tmp_path))
    bad = []
    for key, want in MIN_WAVES.items():
        hits = [(n, v) for n, v in ks.items() if key in n]
        assert hits, "kernel %s not in the library" % key
        for n, v in hits:
            if _waves(v["vgpr"]) < want:
                bad.append("%s: %d registers -> %d waves per SIMD (want >= %d)" % (n, v["vgpr"], _waves(v["vgpr"]), want))
    assert not bad, "\n".join(bad)


def test_single_fit_kernels_use_no_scratch(tmp_path):
    ks = _kernels(str(tmp_path))
    bad = ["%s: %d bytes of scratch" % (n, v["scratch"]) for key in NO_SCRATCH for n, v in ks.items()
           if key in n and v["scratch"] > 0]
    assert not bad, "\n".join(bad)
