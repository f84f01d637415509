"""How far the host runs ahead of the device in the eager C2 step: at the start of each host
step, how many of the previous steps' end events (recorded on the caller's stream after the
join) the device has NOT yet completed.  0 = the device already drained everything the host
enqueued (host-bound); >= 1 = work queued.  Also the host time per step.  Diagnostic only."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from clskd.data import synthetic_pairs  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    kd = bench.build_kd(dev, "step", "mixed")
    Xs, Ys = [], []
    for k in range(bench.NBATCH):
        n, c = synthetic_pairs(bench.B_PER_GPU, bench.L, seed=1000 + k)
        Xs.append(torch.from_numpy(n).to(dev))
        Ys.append(torch.from_numpy(c).to(dev))
    with torch.no_grad():
        for i in range(3):
            kd.training_step((Xs[i % 4], Ys[i % 4]), i)
    torch.cuda.synchronize()
    evs, lead, th = [], [], []
    t0 = time.perf_counter()
    with torch.no_grad():
        for i in range(30):
            pend = sum(1 for e in evs[-8:] if not e.query())
            lead.append(pend)
            a = time.perf_counter()
            kd.training_step((Xs[i % 4], Ys[i % 4]), i)
            th.append(time.perf_counter() - a)
            e = torch.cuda.Event()
            e.record()
            evs.append(e)
    hl = time.perf_counter() - t0
    torch.cuda.synchronize()
    tot = time.perf_counter() - t0
    print("pending steps at each host step start:", lead)
    print(f"host {hl / 30 * 1e3:.3f} ms/step (per-step {min(th) * 1e3:.2f}-{max(th) * 1e3:.2f}), "
          f"device-paced total {tot / 30 * 1e3:.3f} ms/step")


if __name__ == "__main__":
    main()
