"""Build an experiment variant of libredcliff_hip.so with extra -D flags into scripts/bin/ (timing
experiments only, git-ignored but sent to the GPU box; select it with
REDCLIFF_HIP_LIB=scripts/bin/lib_<name>.so)."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))
from redcliff_amd import build as b  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
out = os.path.join(os.path.dirname(__file__), "bin", "lib_%s.so" % name)
os.makedirs(os.path.dirname(out), exist_ok=True)
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=%s" % b.ARCH, "-O3", "-std=c++17", "-fPIC", "-shared", "-I" + b.INCLUDE,
       "-I" + b.CSRC] + flags + b.sources() + ["-o", out]
subprocess.check_call(cmd)
print(os.path.abspath(out))
