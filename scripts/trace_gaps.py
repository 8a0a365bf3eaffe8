"""Busy / idle split of a rocprofv3 kernel trace (the *_kernel_trace.csv of --kernel-trace, or the
*_results.db rocprofv3 writes by default on ROCm 7).

    python scripts/trace_gaps.py TRACE.csv|RESULTS.db [--split-ms 50] [--segment N] [--top 25]

Dispatches are ordered by start time and cut into SEGMENTS at idle gaps longer than --split-ms
(a packed fit's model construction between fits leaves such gaps).  For the chosen segment
(default: the longest) it prints the wall time, the time the device ran at least one kernel, the
idle gaps by size class and the kernels by total time -- the split of a packed fit's wall clock
into kernels and host-side waits.
"""
import argparse
import csv
from collections import defaultdict


def _short(name):
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0]


def load(path):
    if path.endswith(".db"):
        import sqlite3
        con = sqlite3.connect(path)
        rows = [(int(a), int(b), _short(n)) for a, b, n in con.execute("select start, end, name from kernels")]
        rows.sort()
        return rows
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), _short(r["Kernel_Name"])))
    rows.sort()
    return rows


def segments(rows, split_ns):
    segs, cur, end = [], [], None
    for r in rows:
        if cur and r[0] - end > split_ns:
            segs.append(cur)
            cur = []
        cur.append(r)
        end = r[1] if end is None or not cur[:-1] else max(end, r[1])
    if cur:
        segs.append(cur)
    return segs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--split-ms", type=float, default=50.0)
    ap.add_argument("--segment", type=int, default=None)
    ap.add_argument("--top", type=int, default=25)
    args = ap.parse_args()
    segs = segments(load(args.trace), int(args.split_ms * 1e6))
    for i, s in enumerate(segs):
        print("segment %d: %d dispatches, %.2f ms wall, %.2f ms of kernels" % (
            i, len(s), (max(r[1] for r in s) - s[0][0]) / 1e6, sum(r[1] - r[0] for r in s) / 1e6))
    seg = segs[args.segment] if args.segment is not None else max(segs, key=lambda s: max(r[1] for r in s) - s[0][0])
    t0, t1 = seg[0][0], max(r[1] for r in seg)
    busy, end = 0, t0
    gaps = []
    for a, b, _ in seg:
        if a > end:
            gaps.append(a - end)
        busy += max(0, b - max(a, end))
        end = max(end, b)
    wall = t1 - t0
    print("wall %.3f ms, busy %.3f ms (%.1f %%), idle %.3f ms in %d gaps" % (wall / 1e6, busy / 1e6, 100.0 * busy / wall,
                                                                        (wall - busy) / 1e6, len(gaps)))
    for lo, hi in ((0, 5e3), (5e3, 20e3), (20e3, 100e3), (100e3, 1e6), (1e6, 1e12)):
        g = [x for x in gaps if lo <= x < hi]
        print("  gaps %8.0f-%-8.0f us: %5d, %.3f ms" % (lo / 1e3, hi / 1e3, len(g), sum(g) / 1e6))
    per = defaultdict(lambda: [0, 0])
    for a, b, n in seg:
        per[n][0] += 1
        per[n][1] += b - a
    print("%-44s %7s %10s %9s" % ("kernel", "calls", "total ms", "avg us"))
    for n, (cnt, tot) in sorted(per.items(), key=lambda kv: -kv[1][1])[:args.top]:
        print("%-44s %7d %10.3f %9.2f" % (n[:44], cnt, tot / 1e6, tot / cnt / 1e3))


if __name__ == "__main__":
    main()
