"""Per-stream milestones of one eager 3-stream CLSKD step (HIP events recorded on the stream
that reaches each point), relative to the step's first event — the overlap view the rocprof
kernel trace (which serialises streams) cannot give.  Diagnostic only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import clskd.distill as D  # noqa: E402
from clskd.data import synthetic_pairs  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    kd = bench.build_kd(dev, "step", "mixed")
    n, c = synthetic_pairs(bench.B_PER_GPU, bench.L, seed=1)
    X, y = torch.from_numpy(n).to(dev), torch.from_numpy(c).to(dev)
    for _ in range(3):
        kd.training_step((X, y))
    torch.cuda.synchronize()
    runs = []
    for _ in range(5):
        D._MARKS = []
        kd.training_step((X, y))
        kd.training_step((X, y))  # back-to-back like the bench: the next step queued behind
        torch.cuda.synchronize()
        m = D._MARKS[: len(D._MARKS) // 2]
        t0 = m[0][1]
        runs.append([(lab, t0.elapsed_time(ev)) for lab, ev in m])
    D._MARKS = None
    for i, (lab, _) in enumerate(runs[0]):
        vals = sorted(r[i][1] for r in runs)
        print(f"{vals[len(vals) // 2]:8.3f} ms  {lab}")


if __name__ == "__main__":
    main()
