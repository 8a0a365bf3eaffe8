"""Compile libredcliff_hip.so for gfx950 with hipcc (in-tree, so the .so travels with the repo)."""
import glob
import os
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


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _stale(lib=LIB):
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return any(os.path.getmtime(s) > t for s in deps)


def build(force=False, verbose=False, trace=False):
    """Build the HIP shared library if it is missing or older than its sources.
    trace=True builds the phase-timing variant (scripts/phase_trace.py) instead."""
    lib = TRACE_LIB if trace else LIB
    if not force and not _stale(lib):
        return lib
    os.makedirs(LIB_DIR, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, "--offload-arch=%s" % ARCH, "-O3", "-std=c++17", "-fPIC", "-shared", "-I" + INCLUDE, "-I" + CSRC]
    if trace:
        cmd.append("-DRC_TRACE")
    cmd += sources() + ["-o", lib + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    import sys
    print(build(force=True, verbose=True, trace="--trace" in sys.argv))
