"""Repeat the R = 8 matrix-core pack vs independent-fit bitwise check N times in one process
and report each outcome (used to look for the intermittent A mismatch of DESIGN.md §7, v8).

    python scripts/stress_replicas.py [N]        (REDCLIFF_DEFER picks the combine variant)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import pytest  # noqa: E402
import test_gpu_replicas as t  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    bad = 0
    for i in range(n):
        mp = pytest.MonkeyPatch()
        try:
            t.test_packed_replicas_match_independent_fits("mfma", t.GRID8, mp)
            print("iter %d ok" % i, flush=True)
        except AssertionError as e:
            bad += 1
            print("iter %d MISMATCH %s" % (i, str(e).splitlines()[2:4]), flush=True)
        finally:
            mp.undo()
    print("REDCLIFF_DEFER=%s: %d / %d mismatched" % (os.environ.get("REDCLIFF_DEFER", "default"), bad, n))


if __name__ == "__main__":
    main()
