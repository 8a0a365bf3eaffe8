"""Where the time of one data-parallel update goes (one rank over RCCL, TST shape).

    python scripts/dp_profile.py [--batch 128] [--steps 200] [--config c4]

Times N updates of DataParallelFit._step (a) as is, (b) with the all-reduce skipped, and
(c) the host enqueue time alone (the loop returns before the device finishes), next to the
single-fit step of the same shape.  Diagnostic only (no parity claim: (b) skips the collective).
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
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--config", default="c4")
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    import bench
    import redcliff_amd
    from redcliff_amd.data_parallel import DataParallelFit
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(bench._free_port()))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    c = dict(bench.CONFIGS[args.config], B=args.batch)
    B = c["B"]
    model = bench.build_model(redcliff_amd.REDCLIFF_S_CMLP_withStateSmoothing, c, seed=0).to(dev)
    oA, oB = bench.adam_pair(model, c)
    X, Y = bench.synth(c, 16 * B, seed=100)
    dp = DataParallelFit(model, oA, oB)
    ds = dp.cache_dataset([(X[i:i + B], Y[i:i + B]) for i in range(0, X.shape[0], B)])

    def run(n):
        for i in range(n):
            dp._step("combined", ds, i % 16)

    run(20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print("dp step: %.1f us per update (host enqueue %.1f us), %.0f windows/s"
          % (1e6 * t_all / args.steps, 1e6 * t_host / args.steps, args.steps * B / t_all))
    ar = dist.all_reduce
    dist.all_reduce = lambda *a, **k: None
    try:
        run(5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(args.steps)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
    finally:
        dist.all_reduce = ar
    print("dp step without the all-reduce: %.1f us per update" % (1e6 * t / args.steps))
    g = torch.zeros(dp.PA + dp.PB, device=dev)
    for _ in range(10):
        dist.all_reduce(g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dist.all_reduce(g)
    torch.cuda.synchronize()
    print("all_reduce alone (%d floats, 1 rank): %.1f us" % (g.numel(), 1e6 * (time.perf_counter() - t0) / args.steps))
    eng, plan = bench.single_fit(c, args, dev, 0, nbatch=16)
    plan(20, 0).run()
    torch.cuda.synchronize()
    p = plan(args.steps, 20)
    t0 = time.perf_counter()
    p.run()
    torch.cuda.synchronize()
    print("single-fit step (same shape): %.1f us" % (1e6 * (time.perf_counter() - t0) / args.steps))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
