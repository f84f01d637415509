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


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_rccl_communicator_and_allreduce_one_rank():
    """The RCCL path itself (backend "nccl" = RCCL on ROCm) on this box's one GPU: a
    communicator comes up the way clskd.dist.init brings it up (device_id given), the C3
    flat-gradient-sized all-reduce (clskd.train.allreduce_grads' call) and a barrier complete,
    and the result is exact.  (Two ranks cannot share one GPU under RCCL; the world-2 exchange
    is covered over gloo above.)"""
    code = r'''
import os, torch, torch.distributed as dist
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29531")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl"
g = torch.arange(231565, dtype=torch.float32, device="cuda") * 0.5
ref = g.clone()
dist.all_reduce(g, op=dist.ReduceOp.SUM)
dist.barrier()
torch.cuda.synchronize()
assert torch.equal(g, ref)
print("rccl ok", torch.cuda.nccl.version())
dist.destroy_process_group()
'''
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "rccl ok" in r.stdout
