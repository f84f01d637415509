"""Diagnostic (round 6): which tensor of an eager taped forward differs when it runs right after a
TrainStepExecutor capture (before any replay) vs the same forward on a twin model that was never
captured.  Prints the first differing entries of the output tree."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

from clskd.data import synthetic_pairs  # noqa: E402
from clskd.graph import TrainStepExecutor  # noqa: E402
from clskd.train import FlatAdam, FlatParams  # noqa: E402
from test_gpu_parity import _kd  # noqa: E402

DEV = "cuda"
n, c = synthetic_pairs(4, 16000, seed=51)
X, y = torch.from_numpy(n).to(DEV), torch.from_numpy(c).to(DEV)
kd_e, kd_g = _kd().set_precision("mixed"), _kd().set_precision("mixed")
fe, fg = FlatParams(kd_e.student), FlatParams(kd_g.student)
oe, og = FlatAdam(fe, lr=6e-4, device_step=True), FlatAdam(fg, lr=6e-4, device_step=True)
mode = sys.argv[1] if len(sys.argv) > 1 else "capture"
print("mode", mode)
def snap(kd):
    d = {}
    for name, m in kd.named_modules():
        wc = getattr(m, "_wcache", None)
        if isinstance(wc, dict):
            for k, v in wc.items():
                d[("wcache", name, str(k))] = repr(v[0]) if "abfs" in name else repr(
                    [t.data_ptr() if isinstance(t, torch.Tensor) else type(t).__name__
                     for t in (v[1] if isinstance(v[1], (tuple, list)) else [v[1]])])
        fs = m.__dict__.get("_clskd_fold")
        if fs:
            for k, v in fs.items():
                d[("fold", name, str(k))] = (v[0].data_ptr(), int(v[0].abs().sum()), int(v[1].abs().sum()))
    return d


if mode == "capture":
    with torch.no_grad():  # an eager warm-up forward first: caches and fold states exist
        kd_g.forward_with_tape(X, y)
        kd_e.forward_with_tape(X, y)
    torch.cuda.synchronize()
    before = snap(kd_g)
    ex = TrainStepExecutor(kd_g, fg, og, X, y)
    torch.cuda.synchronize()
    after = snap(kd_g)
    for k in sorted(set(before) | set(after)):
        if before.get(k) != after.get(k):
            print("changed", k, before.get(k), "->", after.get(k))
elif mode == "twice":  # no capture: one earlier eager forward on kd_g
    with torch.no_grad():
        kd_g.forward_with_tape(X, y)
elif mode == "twice_e":  # both models run one earlier forward
    with torch.no_grad():
        kd_g.forward_with_tape(X, y)
        kd_e.forward_with_tape(X, y)
elif mode == "step":  # no capture: one earlier eager train step + restore (the capture's warm-up)
    from clskd.graph import _bn_buffers
    state = _bn_buffers(kd_g) + og.state()
    saved = [t.clone() for t in state]
    kd_g.train_step((X, y), fg, og)
    torch.cuda.synchronize()
    with torch.no_grad():
        for t, v in zip(state, saved):
            t.copy_(v)
    fg.bump_versions()
with torch.no_grad():
    a = kd_e.forward_with_tape(X, y)
    b = kd_g.forward_with_tape(X, y)
torch.cuda.synchronize()


def walk(x, y, path, out):
    if isinstance(x, torch.Tensor) and isinstance(y, torch.Tensor):
        if x.shape != y.shape:
            out.append((path, "shape", tuple(x.shape), tuple(y.shape)))
        elif not torch.equal(x, y):
            d = (x.float() - y.float()).abs().max().item()
            out.append((path, "max|diff|", d, x.dtype))
    elif isinstance(x, dict) and isinstance(y, dict):
        for k in x:
            if k in y:
                walk(x[k], y[k], f"{path}.{k}", out)
    elif isinstance(x, (list, tuple)) and isinstance(y, (list, tuple)):
        for i, (u, v) in enumerate(zip(x, y)):
            walk(u, v, f"{path}[{i}]", out)
    elif hasattr(x, "__dict__") and hasattr(y, "__dict__") and type(x) is type(y):
        walk(vars(x), vars(y), path, out)


for k in a:
    o = []
    walk(a[k], b.get(k), k, o)
    print(f"{k:24s} {'DIFF ' + str(len(o)) if o else 'equal'}")
for k, v in a.get("tape", {}).items():
    o = []
    walk(v, b["tape"].get(k), k, o)
    print(f"  tape.{k:18s} {'DIFF ' + str(len(o)) if o else 'equal'}")
out = []
walk(a, b, "out", out)
print(len(out), "differing entries")
for o in out[:60]:
    print(*o)
