"""bench.py's multi-rank plumbing on the CPU (no GPU in the build container): --gpus N without a
launcher starts N ranks itself, the backend reports that world size, and rank 0 prints one JSON
line with n_gpus == N (the driver's SCALE runs rely on this)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _last_json(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


@pytest.mark.parametrize("mode", ["fit", "dp"])
def test_bench_spawns_ranks_itself(mode):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--mode", mode, "--steps", "2",
                        "--warmup", "1"], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 2 and line["config"]["ranks"] == 2 and line["config"]["world_size"] == 2
    devs = line["config"]["rank_devices"]  # every rank's record, all-gathered: distinct processes
    assert [d["rank"] for d in devs] == [0, 1] and [d["local_rank"] for d in devs] == [0, 1]
    assert all(d["device"] == "cpu" for d in devs) and len(set(d["pid"] for d in devs)) == 2
    assert line["scaling"] == ("strong" if mode == "dp" else "weak")
    assert sum(1 for l in r.stdout.splitlines() if l.startswith("{")) == 1  # rank 0 only
