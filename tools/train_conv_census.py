"""Every conv launch of one C3 training step (taped forward, then backward; serialised on one
stream: isolated durations) with its GEMM shape, kernel instance and time, plus totals per
instance and phase.  Diagnostic (round 6: which fp32 launches fall to conv_igemm_f32).

    python tools/train_conv_census.py
"""
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from clskd import ops  # noqa: E402
from clskd.data import synthetic_pairs  # noqa: E402
from clskd.distill import serialized_streams  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    kd = bench.build_kd(dev, "step", "mixed")
    n, c = synthetic_pairs(bench.B_PER_GPU, bench.L, seed=1)
    X, y = torch.from_numpy(n).to(dev), torch.from_numpy(c).to(dev)
    grads = {p: torch.zeros_like(p) for p in kd.student.parameters()}
    tot = collections.defaultdict(lambda: [0, 0.0])
    with torch.no_grad():
        for _ in range(2):
            kd.backward_into(kd.forward_with_tape(X, y), grads)
        torch.cuda.synchronize()
        with serialized_streams():
            ops.KernelTimer.start()
            out = kd.forward_with_tape(X, y)
            torch.cuda.synchronize()
            fwd = ops.KernelTimer.per_launch()
            ops.KernelTimer.stop()
            ops.KernelTimer.start()
            kd.backward_into(out, grads)
            torch.cuda.synchronize()
            bwd = ops.KernelTimer.per_launch()
            ops.KernelTimer.stop()
    for phase, recs in (("fwd", fwd), ("bwd", bwd)):
        print(f"== {phase}")
        for name, shp, us, tf in recs:
            if not any(k in name for k in ("conv", "igemm", "halo", "gemm8", "pointwise", "split")):
                continue
            print(f"{us:8.1f} us {tf:7.1f} TF/s  M={shp[0]:>8} N={shp[1]:>4} K={shp[2]:>5} {shp[3]:4s}  {name}")
            tot[(phase, name)][0] += 1
            tot[(phase, name)][1] += us
    print("totals:")
    for (ph, k), (cnt, us) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{us:9.1f} us {cnt:3d} launches  {ph}  {k}")


if __name__ == "__main__":
    main()
