"""Diagnostic (round 6): tests/test_gpu_train_graph.py::test_train_graph_replays_interleaved_with_
eager_forwards, with cache-clearing toggles — which cache serves the eager forward a stale entry."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

from clskd import config as cfg, ops  # noqa: E402
from clskd.data import synthetic_pairs  # noqa: E402
from clskd.graph import TrainStepExecutor  # noqa: E402
from clskd.model import DCCRN  # noqa: E402
from clskd.train import FlatAdam, FlatParams  # noqa: E402
from test_gpu_parity import _kd  # noqa: E402

DEV = "cuda"
mode = sys.argv[1]
n, c = synthetic_pairs(4, 16000, seed=41)
X, y = torch.from_numpy(n).to(DEV), torch.from_numpy(c).to(DEV)
xe = torch.from_numpy(synthetic_pairs(2, 16000, seed=42)[0]).to(DEV)
kd = _kd().set_precision("mixed")
flat = FlatParams(kd.student)
opt = FlatAdam(flat, lr=6e-4, device_step=True)
ex = TrainStepExecutor(kd, flat, opt, X, y)
for it in range(2):
    ex(X, y)
    torch.cuda.synchronize()
    if mode == "direct":
        ops._DIRECT_W.clear()
    if mode == "wcache":
        kd.student._wcache.clear()
    kd.student.eval()
    with torch.no_grad():
        got = kd.student(xe, is_feat=True).clone()
        fresh = DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT).to(DEV)
        fresh.load_state_dict(kd.student.state_dict())
        fresh.compute = kd.student.compute
        ref = fresh.eval()(xe, is_feat=True)
    kd.student.train()
    torch.cuda.synchronize()
    print(mode, it, "equal" if torch.equal(got, ref) else f"DIFF {(got - ref).abs().max().item():.3e}",
          flush=True)
