"""`bench.py --gpus N` run standalone: the bench starts its own N ranks
(torch.distributed.run as a child process, before anything touches the GPU) and relays rank 0's
line.  Here the two ranks share the one GPU of the box over gloo (test-only overrides
CLSKD_DIST_BACKEND / CLSKD_BENCH_DEVICE); on an 8-GPU node the same command runs one rank per
GPU over RCCL.  The C3 leg is used because it has the one real exchange (the flat gradient
all-reduce): after the timed steps both ranks must hold identical student parameters."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_gpus2_standalone_train_step():
    env = dict(os.environ, CLSKD_DIST_BACKEND="gloo", CLSKD_BENCH_DEVICE="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--train",
                        "--steps", "2", "--warmup", "1"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=560)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["global_batch"] == 2 * d["config"]["per_gpu_batch"]
    h = d["param_hash_per_rank"]
    assert len(h) == 2 and h[0] == h[1], h
