"""Every conv launch of one C2 step (serialised on one stream: isolated durations) with its GEMM
shape, kernel instance and time, in launch order, plus totals per instance.  Diagnostic.

    python tools/conv_census.py [--precision mixed]
"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="mixed")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    kd = bench.build_kd(dev, "step", a.precision)
    n, c = synthetic_pairs(bench.B_PER_GPU, bench.L, seed=1)
    X, y = torch.from_numpy(n).to(dev), torch.from_numpy(c).to(dev)
    with torch.no_grad():
        for _ in range(3):
            kd.training_step((X, y))
        torch.cuda.synchronize()
        ops.KernelTimer.start()
        with serialized_streams():
            kd.training_step((X, y))
        torch.cuda.synchronize()
        recs = ops.KernelTimer.per_launch()
        ops.KernelTimer.stop()
    tot = collections.defaultdict(lambda: [0, 0.0])
    for name, shp, us, tf in recs:
        print(f"{us:8.1f} us {tf:7.1f} TF/s  M={shp[0]:>8} N={shp[1]:>4} K={shp[2]:>5} {shp[3]:4s}  {name}")
        tot[name][0] += 1
        tot[name][1] += us
    print("totals:")
    for k, (cnt, us) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{us:9.1f} us {cnt:3d} launches  {k}")


if __name__ == "__main__":
    main()
