"""Per-step kernel timeline of a rocprofv3 kernel trace (--kernel-trace; *_kernel_trace.csv or
*_results.db): the dispatches of the last --steps steps, each step starting at a dispatch of
--first (default k_forward), with every kernel's start / end relative to the step start and the
idle time before it -- where a single fit's step spends its time between kernels on two streams.

    python scripts/step_timeline.py TRACE [--first k_forward] [--steps 3]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from trace_gaps import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--first", default="k_forward")
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    rows = load(args.trace)  # (start ns, end ns, short name), by start
    starts = [i for i, r in enumerate(rows) if r[2].startswith(args.first)]
    if len(starts) < args.steps + 1:
        sys.exit("fewer than %d steps in the trace" % (args.steps + 1))
    spans = []
    for a, b in zip(starts[-args.steps - 1:-1], starts[-args.steps:]):
        t0 = rows[a][0]
        print("step: %.2f us" % ((rows[b][0] - t0) / 1e3))
        busy_end = t0
        for s, e, n in rows[a:b]:
            idle = max(0, s - busy_end)
            print("  %-34s start %7.2f  end %7.2f  dur %6.2f  idle before %5.2f" %
                  (n[:34], (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, idle / 1e3))
            busy_end = max(busy_end, e)
        spans.append((rows[b][0] - t0) / 1e3)
    print("mean step %.2f us" % (sum(spans) / len(spans)))


if __name__ == "__main__":
    main()
