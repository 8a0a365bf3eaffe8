"""Per-product durations of the GEMM core (k_rc_gemm_mfma / k_rc_gemm) in a rocprofv3 kernel trace
(--kernel-trace --output-format csv): the dispatches grouped by grid shape (one shape per embedder
product of a packed grid step), with the call count, mean / min duration and the grid.

    python scripts/gemm_products.py RUN_kernel_trace.csv [--match k_rc_gemm] [--skip 5]

--skip drops the first N calls of every shape (warm-up steps).
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="k_rc_gemm")
    ap.add_argument("--skip", type=int, default=5)
    args = ap.parse_args()
    by = defaultdict(list)
    order = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            if args.match not in r["Kernel_Name"]:
                continue
            key = (r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0],
                   int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
            if key not in by:
                order.append(key)
            by[key].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    total = 0.0
    for key in order:
        d = [x[1] for x in sorted(by[key])][args.skip:]
        if not d:
            continue
        mean = sum(d) / len(d) / 1e3
        total += mean
        print("%-28s grid %6d x %4d x %5d  calls %4d  mean %8.2f us  min %8.2f us"
              % (key[0], key[1], key[2], key[3], len(d), mean, min(d) / 1e3))
    print("sum of means: %.2f us" % total)


if __name__ == "__main__":
    main()
