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


def _bench2(*extra):
    env = dict(os.environ, CLSKD_DIST_BACKEND="gloo", CLSKD_BENCH_DEVICE="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--steps", "2", "--warmup", "1", *extra],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=560)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["global_batch"] == 2 * d["config"]["per_gpu_batch"]
    return d


@pytest.mark.gpu
@pytest.mark.timeout(1200)
def test_bench_gpus2_standalone_train_step():
    """C3 on two ranks through the same launch path as one rank: the
    captured fwd+loss + backward replayed by the C++ executor, then the flat-gradient all-reduce
    and Adam.  Both ranks end with identical parameters, and they are bitwise the parameters of
    the eager two-rank run (kd.train_step per step) over the same batches.  The ABF modules are
    drawn once (--abf-reinit once): with per-step re-draws the capture's warm-up step advances
    the device draw counter, so the two runs would draw different (equally random) ABF weights."""
    d = _bench2("--train", "--abf-reinit", "once")  # default launch: the executor
    assert d["config"]["launch"].startswith("C++ step executor"), d["config"]["launch"]
    h = d["param_hash_per_rank"]
    assert len(h) == 2 and h[0] == h[1], h
    e = _bench2("--train", "--abf-reinit", "once", "--launch", "eager")
    assert e["config"]["launch"].startswith("eager"), e["config"]["launch"]
    he = e["param_hash_per_rank"]
    assert he[0] == he[1] and he == h, (h, he)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_gpus2_standalone_fwd_loss_executor():
    """The C2 headline leg on two ranks replays the captured step with the executor, as one rank
    does (no exchange in fwd+loss; captured beside the process group's watchdog thread)."""
    d = _bench2()
    assert d["config"]["launch"].startswith("C++ step executor"), d["config"]["launch"]
    assert d["value"] > 0 and d["scaling"] == "weak"


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


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_rccl_process_group_with_captured_train_step():
    """The executor beside an RCCL process group (world 1 on this box's GPU): the training step
    is captured with the communicator and its watchdog thread alive (thread-local capture
    mode), the all-reduce runs between the replay and Adam (TrainStepExecutor collective mode),
    and two replayed steps are bitwise two eager kd.train_step calls (all-reduce + Adam each)."""
    code = r'''
import os, sys, hashlib, torch, torch.distributed as dist
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "speech-enhancement-clskd_amd")]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
import bench
from clskd import config as cfg
from clskd.data import synthetic_pairs
from clskd.graph import TrainStepExecutor
from clskd.train import FlatAdam, FlatParams
xs = []
for k in range(2):
    n, c = synthetic_pairs(4, 16000, seed=70 + k)
    xs.append((torch.from_numpy(n).to(dev), torch.from_numpy(c).to(dev)))
hashes = []
for mode in ("eager", "exec"):
    kd = bench.build_kd(dev, "once", "mixed")
    flat = FlatParams(kd.student)
    opt = FlatAdam(flat, lr=cfg.learning_rate, device_step=True)
    if mode == "exec":
        ex = TrainStepExecutor(kd, flat, opt, xs[0][0], xs[0][1], collective=True)
        assert ex.collective
        for X, Y in xs:
            ex(X, Y)
    else:
        for X, Y in xs:
            kd.train_step((X, Y), flat, opt)
    torch.cuda.synchronize()
    hashes.append(hashlib.sha256(flat.data.cpu().numpy().tobytes()).hexdigest())
    del kd
assert hashes[0] == hashes[1], hashes
print("captured train step with rccl ok")
dist.destroy_process_group()
'''
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, text=True,
                       timeout=560)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "captured train step with rccl ok" in r.stdout
