"""Student fp32 conv shapes (C2 / C3, B=16, T=643): the register-staged split-product engine
(CLSKD_F32X3: conv_split3_kernel), the exact fp32 engine, and the bf16 LDS-DMA engine over
bf16 hi / lo planes with the tripled weight [W_hi | W_hi | W_lo] (+ the planes pass), each with
fused BN statistics where the path supports them.  HIP events over `iters` back-to-back launches.
Diagnostic only (round 6).

    python tools/planes_micro.py [--iters 30]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")]
import torch  # noqa: E402

from clskd import backward as bw  # noqa: E402
from clskd import ops  # noqa: E402
from clskd.ops import OutMap, Seg, SegGeom  # noqa: E402

B, T = 16, 643
# (name, Ci, Co, F_in, kind): student encoder layers (5x2, stride (2,1)) and decoder parities
SHAPES = [("enc3", 32, 64, 32, "enc"), ("enc4", 64, 64, 16, "enc"), ("enc5", 64, 64, 8, "enc"),
          ("dec0p", 128, 64, 4, "dec"), ("dec2p", 128, 32, 16, "dec"), ("dgrad64", 64, 64, 16, "pw3")]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    bw._DGRAD_PLANES = True
    for name, ci, co, fi, kind in SHAPES:
        x = torch.randn(B, fi, T, ci, generator=g).to(dev)
        if kind == "enc":
            taps = [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)]
            Fo, sf = fi // 2, 2
        elif kind == "dec":
            taps = [(dF, -kt) for dF in (1, 0, -1) for kt in (0, 1)]
            Fo, sf = fi, 1
        else:
            taps = [(kf - 1, kt - 1) for kf in range(3) for kt in range(2)]
            Fo, sf = fi, 1
        K = len(taps) * ci
        wt = ops.pack_weight((torch.randn(co, len(taps), ci, generator=g) * 0.05).to(dev), K)
        out = torch.empty(B, Fo, T, co, device=dev)
        omap = OutMap(Fo * T * co, T * co, co)
        geom = SegGeom(ci, fi * T * ci, T * ci, ci, fi, T)
        seg = Seg(x, 0, geom)
        nblk = ops.conv_mblocks(B, Fo, T)
        st = torch.empty(nblk * co * 2, device=dev, dtype=torch.float64)

        def split3():
            with ops.split_products(True):
                ops.conv([seg], taps, B, Fo, T, co, wt, None, out, omap, stride_f=sf, stats=st)

        def exact():
            ops.conv([seg], taps, B, Fo, T, co, wt, None, out, omap, stride_f=sf, stats=st,
                     mfma_only=True)
        planes, segs = bw._planes_of(x, geom)
        w3 = bw._split3_weight(wt, len(taps), ci)

        def planes_conv():
            ops.conv(segs, taps, B, Fo, T, co, w3, None, out, omap, stride_f=sf, stats=st)

        def planes_all():
            ops.split_planes(x, planes)
            planes_conv()
        res = {k: timeit(f, a.iters) for k, f in (("split3", split3), ("exact", exact),
                                                  ("planes_conv", planes_conv),
                                                  ("planes+split", planes_all))}
        ops.conv([seg], taps, B, Fo, T, co, wt, None, out, omap, stride_f=sf, stats=st)
        names = ""
        M = B * Fo * T
        print(f"{name:8s} M={M:8d} N={co:3d} K={K:5d}  " +
              "  ".join(f"{k} {v:7.1f} us" for k, v in res.items()) + names, flush=True)


if __name__ == "__main__":
    main()
