"""North-star config (C1, K=4) single-fit step time with and without an RCCL process group in the
process, and with the split-lead step on / off (REDCLIFF_SPLIT_LEAD, read by the library per call).

    python scripts/ns_probe.py [--config c1k4] [--nccl]
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
    ap.add_argument("--config", default="c1k4")
    ap.add_argument("--nccl", action="store_true", help="create a one-rank nccl (RCCL) process group first")
    args = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if args.nccl:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(bench._free_port()))
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        t = torch.ones(1, device=dev)
        dist.all_reduce(t)
    c = bench.CONFIGS[args.config]
    _, plan = bench.single_fit(c, args, dev, 0)
    plan(5, 0).run()
    start = 5 + bench.preheat(plan, 5, 0.3)
    for split in ("auto", "0", "1", "auto"):
        if split == "auto":
            os.environ.pop("REDCLIFF_SPLIT_LEAD", None)
        else:
            os.environ["REDCLIFF_SPLIT_LEAD"] = split
        plan(20, start).run()
        el = bench.timed(plan(100, start + 20).run, None, dev)
        start += 120
        print(json.dumps({"config": args.config, "nccl": args.nccl, "split_lead": split,
                          "ms_per_step": round(1e3 * el / 100, 5), "windows_per_s": round(100 * c["B"] / el, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
