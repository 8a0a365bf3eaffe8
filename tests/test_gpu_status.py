"""Device status of the merged backward's producer/consumer hand-off (rc_common.h rc_wait_count):
a consumer whose poll runs out counts itself into its replica's status word instead of
carrying on silently; the host reads the word (redcliff_device_status / the fit's per-epoch
copy back) and raises.  REDCLIFF_DEBUG_WAIT_TIMEOUT=1 makes every consumer wait for one
producer more than exists (short poll bound), which forces that path.  Also: the vector
factor backward's LDS limit is reported with the batch size that fits."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from test_gpu_replicas import data, make, opts

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "redcliff-s-hypothesizing-dynamic-causal-graphs_amd")

CHILD = r"""
import sys
sys.path.insert(0, %(root)r); sys.path.insert(0, %(pkg)r); sys.path.insert(0, %(tests)r)
import torch
from test_gpu_replicas import data, make, opts
m = make(0, 10.0, 0.1)
oA, oB = opts(m, 5e-4, 2e-4)
X, Y = data(64, seed=3)[0]
m.batch_update(2, 0, X, Y, oA, oB, 1)     # combined phase: the merged backward (D4IC, single fit)
torch.cuda.synchronize()
try:
    m.check_device_status()
except RuntimeError as e:
    assert "timed out" in str(e), str(e)
    m.check_device_status()                # the word was cleared by the first check
    print("RAISED", flush=True)
else:
    print("SILENT", flush=True)
train, val = data(64 * 2, seed=4), data(64, seed=5)
try:
    m.fit(None, train, oA, oB, 4, 1, 1, 4, val, lookback=1, check_every=1, verbose=0)
except RuntimeError as e:
    assert "timed out" in str(e), str(e)
    print("FIT RAISED", flush=True)
"""


def test_forced_wait_timeout_is_reported():
    env = dict(os.environ, REDCLIFF_DEBUG_WAIT_TIMEOUT="1", REDCLIFF_MERGE="1")
    code = CHILD % dict(root=ROOT, pkg=PKG, tests=os.path.join(ROOT, "tests"))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "RAISED" in out.stdout and "FIT RAISED" in out.stdout, out.stdout + out.stderr[-2000:]


def test_status_clean_after_normal_steps():
    from redcliff_amd import _native as nat
    m = make(0, 10.0, 0.1)
    oA, oB = opts(m, 5e-4, 2e-4)
    for bi, (X, Y) in enumerate(data(128, seed=3)):
        m.batch_update(2, bi, X, Y, oA, oB, 1)
    eng = m.engine()
    d = eng.dims(eng.ws_dims[0], 21)
    words = nat.device_status(d, eng.ws.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert words == [0], words
    m.check_device_status()


def test_vector_factor_path_names_its_batch_limit(monkeypatch):
    """REDCLIFF_FAC_PATH=vector on a batch whose per-window LDS tiles exceed 64 KiB: a clear
    ELIMIT naming the largest batch that fits (the default path switches to the matrix cores)."""
    from test_gpu_data_parallel import CFG as TST, _model
    monkeypatch.setenv("REDCLIFF_FAC_PATH", "vector")
    m, oA, oB = _model()  # TST shape: K = 9 factors, 512 windows (the configs[3] large-shard case)
    rng = np.random.RandomState(0)
    X = torch.from_numpy(rng.randn(512, TST["T"], TST["p"]).astype(np.float32))
    Y = torch.zeros(512, TST["K"], TST["T"])
    Y[:, 0] = 1.0
    with pytest.raises(RuntimeError, match="use batches of at most"):
        m.batch_update(2, 0, X, Y, oA, oB, 1)
