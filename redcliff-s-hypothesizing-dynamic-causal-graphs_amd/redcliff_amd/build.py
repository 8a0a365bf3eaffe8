"""Compile libredcliff_hip.so for gfx950 with hipcc (in-tree, so the .so travels with the repo).

Every build compiles ``source_hash`` (SHA-256 over the kernel sources, the public header and
the compile defines) into the library as ``redcliff_build_id()``; a library is current when its
embedded id equals the hash of the tree it sits in, not when its mtime is newer."""
import glob
import hashlib
import os
import re
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
REPO_ROOT = os.path.dirname(PKG_ROOT)
CSRC = os.path.join(PKG_ROOT, "csrc")
INCLUDE = os.path.join(REPO_ROOT, "include")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libredcliff_hip.so")
TRACE_LIB = os.path.join(LIB_DIR, "libredcliff_hip_trace.so")  # -DRC_TRACE: per-phase wall-clock marks
ARCH = os.environ.get("REDCLIFF_OFFLOAD_ARCH", "gfx950")
# Diagnostic variants (scripts/race_probe.py): the round-1 A-mismatch race made reproducible by
# delaying waves >= 1 of k_emb_final's adjacency workgroup, with and without the fixing barrier.
VARIANTS = {
    "probe_fixed": ["-DRC_PROBE_DELAY"],
    "probe_nobarrier": ["-DRC_PROBE_DELAY", "-DRC_PROBE_NO_BARRIER"],
}


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def variant_path(name):
    return os.path.join(LIB_DIR, "libredcliff_hip_%s.so" % name)


def source_files():
    return sorted(sources() + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h")))


def source_hash(defines=()):
    """First 16 hex digits of SHA-256 over (relative path, contents) of every source the library is
    compiled from, the offload arch and the extra -D flags (so variants get their own id)."""
    h = hashlib.sha256()
    for path in source_files():
        rel = os.path.relpath(path, REPO_ROOT).replace(os.sep, "/")
        with open(path, "rb") as f:
            data = f.read()
        h.update(rel.encode() + b"\0" + str(len(data)).encode() + b"\0" + data)
    h.update(("arch=%s;defines=%s" % (ARCH, " ".join(defines))).encode())
    return h.hexdigest()[:16]


_TAG = re.compile(rb"REDCLIFF_BUILD_ID=([0-9a-f]{16})")


def embedded_id(lib=LIB):
    """The build id compiled into `lib` (read from the file bytes; the library is not loaded),
    or None when the file is missing or carries no id."""
    try:
        with open(lib, "rb") as f:
            m = _TAG.search(f.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def _stale(lib=LIB, defines=()):
    return embedded_id(lib) != source_hash(defines)


def _compile(lib, defines, verbose):
    """One object per translation unit, compiled in parallel, then one link."""
    from concurrent.futures import ThreadPoolExecutor
    import tempfile
    os.makedirs(LIB_DIR, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    bid = '-DREDCLIFF_BUILD_ID="%s"' % source_hash(defines)
    base = [hipcc, "--offload-arch=%s" % ARCH, "-O3", "-std=c++17", "-fPIC", "-I" + INCLUDE, "-I" + CSRC, bid] + list(defines)
    with tempfile.TemporaryDirectory(prefix="rc_build_") as tmp:
        objs = [os.path.join(tmp, os.path.basename(s) + ".o") for s in sources()]
        cmds = [base + ["-c", s, "-o", o] for s, o in zip(sources(), objs)]
        jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
        with ThreadPoolExecutor(jobs) as ex:
            for cmd in cmds:
                if verbose:
                    print(" ".join(cmd))
            list(ex.map(subprocess.check_call, cmds))
        # -Bsymbolic: the library's own calls bind inside it, so a diagnostic variant can be loaded
        # next to the production library without either resolving into the other
        link = [hipcc, "--offload-arch=%s" % ARCH, "-shared", "-fPIC", "-Wl,-Bsymbolic"] + objs + ["-o", lib + ".tmp"]
        if verbose:
            print(" ".join(link))
        subprocess.check_call(link)
    os.replace(lib + ".tmp", lib)
    return lib


def build(force=False, verbose=False, trace=False):
    """Build the HIP shared library if it is missing or older than its sources.
    trace=True builds the phase-timing variant (scripts/phase_trace.py) instead."""
    lib = TRACE_LIB if trace else LIB
    defines = ["-DRC_TRACE"] if trace else []
    if not force and not _stale(lib, defines):
        return lib
    return _compile(lib, defines, verbose)


def build_variant(name, force=False, verbose=False):
    """Build one of the diagnostic VARIANTS (not part of the product)."""
    lib = variant_path(name)
    if not force and not _stale(lib, VARIANTS[name]):
        return lib
    return _compile(lib, VARIANTS[name], verbose)


if __name__ == "__main__":
    import sys
    if "--variants" in sys.argv:
        for v in VARIANTS:
            print(build_variant(v, force=True, verbose=True))
    else:
        print(build(force=True, verbose=True, trace="--trace" in sys.argv))
