"""Why a 20-step timed region reads slower than a 300-step one (VERDICT r3 "What's weak" #1).

    python scripts/steady_state.py [--config d4ic]

Builds bench.py's single fit, then times back-to-back regions of the bench's kind (barrier-free,
synchronize on both sides) in several situations and prints one JSON line per measurement:
  * 20-step regions right after a 5-step warm-up, repeated (does the first one differ?);
  * per-step device times of one 20-step region (events between one-step launches);
  * 20 steps after the device idled for 1 s (clock / power ramp after idle);
  * 20 steps right after 0.3 s of back-to-back steps;
  * one 300-step region.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="d4ic")
    args = ap.parse_args()
    import torch
    import bench
    c = bench.CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng, plan = bench.single_fit(c, args, dev, 0)
    B = c["B"]

    def region(n, start):
        p = plan(n, start)
        el = bench.timed(p.run, None, dev)
        return 1e3 * el / n

    def emit(what, ms):
        print(json.dumps({"what": what, "ms_per_step": round(ms, 5), "windows_per_s": round(B / ms * 1e3, 1)}),
              flush=True)

    plan(5, 0).run()
    for i in range(4):
        emit("20-step region #%d after 5-step warm-up" % i, region(20, 5 + 20 * i))
    # per-step device time of one region: one launch per step, events between them
    plans = [plan(1, 100 + i) for i in range(20)]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
    torch.cuda.synchronize()
    ev[0].record()
    for i, p in enumerate(plans):
        p.run()
        ev[i + 1].record()
    torch.cuda.synchronize()
    per = [ev[i].elapsed_time(ev[i + 1]) for i in range(20)]
    print(json.dumps({"what": "per-step device ms, one-step launches", "ms": [round(x, 4) for x in per]}), flush=True)
    time.sleep(1.0)
    emit("20 steps after 1 s idle", region(20, 200))
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 0.3:
        plan(50, n).run()
        torch.cuda.synchronize()
        n += 50
    emit("20 steps right after 0.3 s of steps", region(20, 300))
    emit("300-step region", region(300, 400))
    emit("20 steps right after 300", region(20, 700))
    time.sleep(1.0)
    emit("20 steps after another 1 s idle", region(20, 800))


if __name__ == "__main__":
    main()
