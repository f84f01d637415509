"""Host-side enqueue time of one eager CLSKD step (no device sync inside), vs device time."""
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
    kd = bench.build_kd(dev, "step", "mixed")
    n, c = synthetic_pairs(bench.B_PER_GPU, bench.L, seed=1)
    X, y = torch.from_numpy(n).to(dev), torch.from_numpy(c).to(dev)
    for _ in range(3):
        kd.training_step((X, y))
    torch.cuda.synchronize()
    hs = []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kd.training_step((X, y))
        hs.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    print(f"host enqueue per step: min {min(hs) * 1e3:.2f} ms, median {sorted(hs)[5] * 1e3:.2f} ms")


if __name__ == "__main__":
    main()
