"""Does a HIP graph of the single-fit step chain run faster than the stream launches?  (Timing probe
only: a replayed graph reuses the captured Adam step numbers, so its parameters are not a valid
fit -- the question is the per-step time of the same launch chain.)

    python scripts/graph_probe.py [--config d4ic] [--steps 20]
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
    ap.add_argument("--config", default="d4ic")
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c = bench.CONFIGS[args.config]
    _, plan = bench.single_fit(c, args, dev, 0)
    plan(5, 0).run()
    start = 5 + bench.preheat(plan, 5, 0.3)
    n = args.steps
    el = bench.timed(plan(n, start).run, None, dev)
    el300 = bench.timed(plan(300, start + n).run, None, dev)
    # capture n steps on a side stream (torch's graph capture), then replay
    p = plan(n, start + n + 300)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            p.run()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    elg = bench.timed(g.replay, None, dev)

    def many():
        for _ in range(15):
            g.replay()
    elg15 = bench.timed(many, None, dev)
    print(json.dumps({"config": args.config, "steps": n, "stream_ms_per_step": round(1e3 * el / n, 5),
                      "stream_300_ms_per_step": round(1e3 * el300 / 300, 5),
                      "graph_ms_per_step": round(1e3 * elg / n, 5),
                      "graph_15x_ms_per_step": round(1e3 * elg15 / (15 * n), 5)}), flush=True)


if __name__ == "__main__":
    main()
