"""Packed grid-search steps only (the bench's grid_search leg without the rest), for rocprofv3
kernel traces and counter passes.

    python scripts/grid_step.py [--replicas 128] [--steps 20] [--config d4ic]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=128)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--config", default="d4ic")
    args = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c = bench.CONFIGS[args.config]
    ns = argparse.Namespace(replicas=args.replicas, grid_steps=args.steps)
    el, R, steps = bench.run_grid(c, ns, dev, 0, None)
    print("grid R=%d: %.4f ms per step, %.0f windows/s" % (R, 1e3 * el / args.steps, R * args.steps * c["B"] / el))
    t0 = time.perf_counter()
    steps(args.steps, 3)()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print("grid R=%d (again): %.4f ms per step" % (R, 1e3 * el / args.steps))


if __name__ == "__main__":
    main()
