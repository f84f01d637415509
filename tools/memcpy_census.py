"""Which torch calls record memcpy nodes in the captured C3 training step (diagnostic): wraps
Tensor.clone / copy_ / contiguous / to / torch.clone / torch.cat and counts, by caller file:line,
the calls made while a capture is active that copy a contiguous tensor into a contiguous one of
the same dtype (the D2D copies torch issues as memcpys).

    python tools/memcpy_census.py
"""
import collections
import os
import sys
import traceback

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                             "speech-enhancement-clskd_amd")]
import torch  # noqa: E402

CNT = collections.Counter()


def site():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if "clskd" in fr.filename or "bench" in fr.filename:
            return f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.line}"
    return "?"


def wrap(owner, name):
    orig = getattr(owner, name)

    def w(*a, **k):
        if torch.cuda.is_current_stream_capturing():
            CNT[f"{name} @ {site()}"] += 1
        return orig(*a, **k)
    setattr(owner, name, w)


def main():
    from clskd.data import synthetic_pairs
    from clskd.graph import TrainStepGraph
    from clskd.train import FlatAdam, FlatParams
    from test_gpu_parity import _kd
    n, c = synthetic_pairs(4, 16000, seed=31)
    X, y = torch.from_numpy(n).cuda(), torch.from_numpy(c).cuda()
    kd = _kd().set_precision("mixed")
    flat = FlatParams(kd.student)
    opt = FlatAdam(flat, lr=6e-4, device_step=True)
    for name in ("clone", "copy_", "contiguous", "to", "reshape", "flatten", "float", "view"):
        wrap(torch.Tensor, name)
    for name in ("clone", "cat", "stack"):
        wrap(torch, name)
    TrainStepGraph(kd, flat, opt, X, y)
    for k, v in CNT.most_common():
        print(f"{v:4d}  {k}")


if __name__ == "__main__":
    main()
