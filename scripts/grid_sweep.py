"""Packed grid step (R replicas, bench.py's grid leg) under the library's tuning knobs, one
process, interleaved settings: which launch-shape choices are best at this R.

    python scripts/grid_sweep.py [--replicas 128] [--steps 40] [--rounds 2]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))

SETTINGS = [
    {},
    {"REDCLIFF_FORK": "1"},
    {"REDCLIFF_EMB_FINAL_EPT": "1"},
    {"REDCLIFF_EMB_FINAL_EPT": "2"},
    {"REDCLIFF_EMB_FINAL_EPT": "8"},
    {"REDCLIFF_FAC_BPW": "1"},
    {"REDCLIFF_FAC_BPW": "2"},
    {"REDCLIFF_GEMM_TILE": "32"},
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=128)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--config", default="d4ic")
    ap.add_argument("--settings", default=None, help="JSON list of environment dicts (default: the built-in list)")
    ap.add_argument("--kernel-times", action="store_true",
                    help="also the per-kernel HIP-event averages (us) of each setting (10 more steps)")
    args = ap.parse_args()
    settings = json.loads(args.settings) if args.settings else SETTINGS
    knobs = sorted(set(k for st in settings for k in st))
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c = bench.CONFIGS[args.config]
    ns = argparse.Namespace(replicas=args.replicas, grid_steps=args.steps)
    _, R, steps = bench.run_grid(c, ns, dev, 0, None)
    start = 10
    for rnd in range(args.rounds):
        for st in settings:
            for k in knobs:
                os.environ.pop(k, None)
            os.environ.update(st)
            steps(5, start)()
            el = bench.timed(steps(args.steps, start + 5), None, dev)
            start += 5 + args.steps
            rec = {"replicas": R, "round": rnd, "setting": st, "ms_per_step": round(1e3 * el / args.steps, 4),
                   "windows_per_s": round(R * args.steps * c["B"] / el, 1)}
            if args.kernel_times:
                kt = bench.kernel_times_of(steps(10, start))
                start += 10
                rec["kernel_us"] = dict((k, round(v[0] * 1e3, 2)) for k, v in kt.items() if v[1])
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
