"""Single-fit step time of one library build (A/B runs: select the build with REDCLIFF_HIP_LIB).

    REDCLIFF_HIP_LIB=scripts/bin/lib_prev.so python scripts/ab_single.py --tag prev [--configs d4ic,c1k4,c4]

Per config: bench.py's single fit, warm-up + preheat, then a 20-step region (the driver's) and a
300-step region; one JSON line each.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default=os.environ.get("REDCLIFF_HIP_LIB", "tree"))
    ap.add_argument("--configs", default="d4ic,c1k4,c4")
    args = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for name in args.configs.split(","):
        c = bench.CONFIGS[name]
        _, plan = bench.single_fit(c, args, dev, 0)
        plan(5, 0).run()
        start = 5 + bench.preheat(plan, 5, 0.3)
        el20 = bench.timed(plan(20, start).run, None, dev)
        el300 = bench.timed(plan(300, start + 20).run, None, dev)
        print(json.dumps({"tag": args.tag, "config": name, "ms_20": round(1e3 * el20 / 20, 5),
                          "ms_300": round(1e3 * el300 / 300, 5), "windows_per_s_300": round(300 * c["B"] / el300, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
