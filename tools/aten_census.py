"""Census of the PyTorch (aten) ops the C2 step dispatches besides the library's own kernels —
every one is a launch (elementwise, cat, copy) that the host enqueues and the device runs.
Counts ops per step by (op, innermost clskd source line).  Diagnostic only.
    python tools/aten_census.py [steps]"""
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")]

# metadata-only ops: no launch
_FREE = {"empty", "empty_strided", "view", "_unsafe_view", "reshape", "as_strided", "t", "transpose",
         "permute", "select", "slice", "unsqueeze", "squeeze", "expand", "detach", "alias", "split",
         "unbind", "chunk", "narrow", "lift_fresh", "_to_copy_noop", "set_", "record_stream",
         "is_same_size", "new_empty", "new_empty_strided", "empty_like", "split_with_sizes", "_local_scalar_dense"}


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.overloadpacket.__name__
        if name not in _FREE:
            where = "?"
            for fr in reversed(traceback.extract_stack(limit=30)):
                if "clskd" in fr.filename and "aten_census" not in fr.filename:
                    where = f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.name}"
                    break
            self.c[(name, where)] += 1
        return func(*args, **(kwargs or {}))


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    import bench
    from clskd.data import synthetic_pairs
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    kd = bench.build_kd(dev, "step", os.environ.get("PRECISION", "mixed"))
    Xs, Ys = [], []
    for k in range(2):
        noisy, clean = synthetic_pairs(bench.B_PER_GPU, bench.L, seed=1000 + k)
        Xs.append(torch.from_numpy(noisy).to(dev))
        Ys.append(torch.from_numpy(clean).to(dev))
    if os.environ.get("TRAIN") == "1":  # the C3 training step (bench.py --train's eager step)
        from clskd import config as cfg
        from clskd.train import FlatAdam, FlatParams
        flat = FlatParams(kd.student)
        opt = FlatAdam(flat, lr=cfg.learning_rate, device_step=True)
        step = lambda i: kd.train_step((Xs[i % 2], Ys[i % 2]), flat, opt)
    else:
        step = lambda i: kd.training_step((Xs[i % 2], Ys[i % 2]), i)
    with torch.no_grad():
        for i in range(3):
            step(i)
        torch.cuda.synchronize()
        cen = Census()
        with cen:
            for i in range(steps):
                step(i)
        torch.cuda.synchronize()
    tot = sum(cen.c.values())
    print(f"aten ops per step: {tot / steps:.1f}")
    for (name, where), n in cen.c.most_common():
        print(f"{n / steps:6.1f}  {name:28s} {where}")


if __name__ == "__main__":
    main()
