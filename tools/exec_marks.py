"""Per-stream end times of one C2 step, eager four-stream launch vs the C++ executor replaying the
captured step (HIP timing events; diagnostic).  Eager: tools/stream_marks.py's milestones (events
recorded on the stream that reaches each point); executor: clskd_exec_marks (an event before the
fork and at every stream's tail).  Steps run back to back as in the bench.

    python tools/exec_marks.py [steps]
"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import clskd.distill as D  # noqa: E402
from clskd import _lib  # noqa: E402
from clskd.data import synthetic_pairs  # noqa: E402
from clskd.graph import StepExecutor  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    kd = bench.build_kd(dev, "step", "mixed")
    n, c = synthetic_pairs(bench.B_PER_GPU, bench.L, seed=1)
    X, y = torch.from_numpy(n).to(dev), torch.from_numpy(c).to(dev)
    ex = StepExecutor(kd, X, y)
    for _ in range(3):
        with torch.no_grad():
            kd.training_step((X, y))
    torch.cuda.synchronize()
    # eager: milestone events, steps back to back
    runs = []
    for _ in range(5):
        D._MARKS = []
        with torch.no_grad():
            for _ in range(3):
                kd.training_step((X, y))
        torch.cuda.synchronize()
        m = D._MARKS
        per = len(m) // 3
        mid = m[per:2 * per]  # the middle step: queued behind one, ahead of one
        t0 = mid[0][1]
        runs.append([(lab, t0.elapsed_time(ev)) for lab, ev in mid])
    D._MARKS = None
    print("eager milestones (median of 5, ms after the step's first event):")
    for i, (lab, _) in enumerate(runs[0]):
        vals = sorted(r[i][1] for r in runs)
        print(f"  {vals[len(vals) // 2]:8.3f}  {lab}")
    # executor
    lib = _lib.load()
    for _ in range(3):
        ex(X, y)
    torch.cuda.synchronize()
    _lib.check(lib.clskd_exec_marks(ex._ex, 1), "marks")
    torch.cuda.synchronize()
    for _ in range(steps):
        ex(X, y)
    torch.cuda.synchronize()
    out = (C.c_float * 8)()
    _lib.check(lib.clskd_exec_marks_read(ex._ex, out, 8), "marks_read")
    names = ["0 caller (grams, ReviewKD-dec, join)", "1 student", "2 ReviewKD-enc / MRSTFT", "3 teacher"]
    print(f"executor stream tails (mean over {steps} back-to-back replays, ms after the fork):")
    for s in range(ex.nstreams):
        print(f"  {out[s]:8.3f}  {names[s] if s < len(names) else s}")
    print("executor info:", ex.info)


if __name__ == "__main__":
    main()
