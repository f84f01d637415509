"""Per-launch census of the conv engine over one eager CLSKD step (bench workload C2):
kernel variant, GEMM shape (M = B*Fo*To, N, K), duration and TFLOP/s.  Diagnostic only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from clskd import ops  # noqa: E402
from clskd.data import synthetic_pairs  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    kd = bench.build_kd(dev, "step", sys.argv[1] if len(sys.argv) > 1 else "mixed")
    n, c = synthetic_pairs(bench.B_PER_GPU, bench.L, seed=1)
    X, y = torch.from_numpy(n).to(dev), torch.from_numpy(c).to(dev)
    for _ in range(2):
        kd.training_step((X, y))
    torch.cuda.synchronize()
    # serialise the three streams so per-launch times are not inflated by overlap
    import clskd.distill as D
    for which in (0, 1):
        D._SIDE[(dev.index, which)] = torch.cuda.current_stream(dev)
    ops.KernelTimer.start()
    kd.training_step((X, y))
    torch.cuda.synchronize()
    recs = ops.KernelTimer.per_launch()
    ops.KernelTimer.stop()
    tot = 0.0
    print(f"{'kernel':46s} {'M':>9s} {'N':>5s} {'K':>6s} {'dt':>5s} {'us':>8s} {'TF/s':>7s}")
    for name, (M, N, K, dt), us, tf in recs:
        tot += us
        print(f"{name:46s} {M:9d} {N:5d} {K:6d} {dt:>5s} {us:8.1f} {tf:7.1f}")
    print(f"total {tot / 1e3:.3f} ms over {len(recs)} launches")


if __name__ == "__main__":
    main()
