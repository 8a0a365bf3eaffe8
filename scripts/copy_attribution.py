"""Which device copies (``__amd_rocclr_copyBuffer``, the blit kernel behind hipMemcpy*) fall inside
the timed packed fit of bench.py's fits/hour leg, and which are setup (model construction / binding,
data upload, the warm-up copy of the pack)?

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ca -o run -- python scripts/copy_attribution.py
    python scripts/copy_attribution.py --parse gpurun_out/ca/.../run_kernel_trace.csv > profiles/r05_copy_attribution.json

The timed fit is bracketed by two ``torch.cuda._sleep`` launches (kernel name contains "sleep" /
"spin"); --parse counts every kernel by name before, inside and after that bracket."""
import argparse
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd"))


def run(args):
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c = bench.CONFIGS["d4ic"]
    ns = argparse.Namespace(fit_replicas=args.replicas, fit_epochs=args.epochs, fit_train_batches=8)
    marks = []
    orig = bench.timed

    def timed(fn, dist, dev_):  # the fits/hour leg's timed region, bracketed by marker kernels
        torch.cuda.synchronize()
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
        el = orig(fn, dist, dev_)
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
        marks.append(el)
        return el
    bench.timed = timed
    out = bench.fits_per_hour(c, ns, dev, 0, None, 1)
    print(json.dumps({"fits_per_hour": out["value"], "timed_seconds": marks}), flush=True)


def parse(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    mk = [i for i, (_, _, n) in enumerate(rows) if "sleep" in n.lower() or "spin" in n.lower()]
    assert len(mk) >= 2, "marker kernels not found"
    a, b = mk[-2], mk[-1]
    parts = {"before_timed_fit": rows[:a], "timed_fit": rows[a + 1:b], "after": rows[b + 1:]}
    out = {}
    for k, rs in parts.items():
        cnt, dur = {}, {}
        for s, e, n in rs:
            key = n if len(n) < 90 else n[:90]
            cnt[key] = cnt.get(key, 0) + 1
            dur[key] = dur.get(key, 0) + (e - s)
        top = sorted(cnt, key=lambda n: -dur[n])[:12]
        out[k] = {"kernels": len(rs), "copyBuffer_calls": sum(v for n, v in cnt.items() if "copyBuffer" in n),
                  "copyBuffer_ms": round(sum(v for n, v in dur.items() if "copyBuffer" in n) / 1e6, 3),
                  "wall_ms": round((rs[-1][1] - rs[0][0]) / 1e6, 3) if rs else 0.0,
                  "top_by_time": [{"kernel": n, "calls": cnt[n], "ms": round(dur[n] / 1e6, 3)} for n in top]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--parse", default=None)
    ap.add_argument("--replicas", type=int, default=128)
    ap.add_argument("--epochs", type=int, default=40)
    a = ap.parse_args()
    if a.parse:
        parse(a.parse)
    else:
        run(a)
