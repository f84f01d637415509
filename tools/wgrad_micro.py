"""Weight-gradient microbenchmark on the C3 student's shapes (B=16, T=643/644: the layers of
tools/bwd_census.py): the exact fp32 engine (conv_wgrad_f32) against the split-product engine
(csrc/wgrad_x3.hip, one / two chunks in flight per wave and the default per-instance pick:
CLSKD_WGRAD_DEPTH 1 / 2 / 0), `iters`
back-to-back launches timed with HIP events.  Diagnostic only.

    python tools/wgrad_micro.py [--iters 20] [--only n2_k96,n8_k20]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")]
import torch  # noqa: E402

from clskd import ops  # noqa: E402

ENC = [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)]
DEC = [(dF, -kt) for dF in (1, 0, -1) for kt in (0, 1)]
CASES = {
    # name: (segment channels, N, taps, stride_f, Fi, Fo, T)
    "n2_k96": ((8, 8), 2, DEC, 1, 128, 128, 644),
    "n8_k20": ((2,), 8, ENC, 2, 256, 128, 643),
    "n8_k192": ((16, 16), 8, DEC, 1, 64, 64, 644),
    "n16_k80": ((8,), 16, ENC, 2, 128, 64, 643),
    "n16_k384": ((32, 32), 16, DEC, 1, 32, 32, 644),
    "n32_k160": ((16,), 32, ENC, 2, 64, 32, 643),
    "n32_k768": ((64, 64), 32, DEC, 1, 16, 16, 644),
    "n64_k320": ((32,), 64, ENC, 2, 32, 16, 643),
    "n64_k768": ((64, 64), 64, DEC, 1, 8, 8, 644),
    "n128_k32": ((32,), 128, [(0, 0)], 1, 1, 1, 1286),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--B", type=int, default=16)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    names = [n for n in CASES if not args.only or n in args.only.split(",")]
    from clskd import _lib
    legs = [("f32", False, 0), ("x3d1", True, 1), ("x3d2", True, 2), ("x3", True, 0)]
    tot = {lg[0]: 0.0 for lg in legs}
    for name in names:
        segc, N, taps, sf, Fi, Fo, T = CASES[name]
        B = args.B
        g = torch.Generator().manual_seed(0)
        segs = [ops.seg_bftc(torch.randn(B, Fi, T, c, generator=g).to(dev)) for c in segc]
        dy = torch.randn(B, Fo, T, N, generator=g).to(dev)
        K = len(taps) * sum(segc)
        Kp = -(-K // 16) * 16
        dw = torch.empty(N, Kp, device=dev)
        db = torch.empty(N, device=dev)
        om = ops.OutMap(Fo * T * N, T * N, N)
        row = []
        for leg, split, depth in legs:
            _lib.set_knob("CLSKD_WGRAD_DEPTH", depth)

            def run():
                with ops.split_products(False, wgrad=split):
                    ops.conv_wgrad(segs, taps, B, Fo, T, N, dy, om, dw, db, stride_f=sf)
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            tot[leg] += us
            row.append(f"{leg} {us:8.1f} us {2.0 * B * Fo * T * N * K / us / 1e6:6.1f} TF/s")
        print(f"{name:10s} M={B * Fo * T:8d} N={N:4d} K={K:5d}  " + "  ".join(row), flush=True)
    _lib.set_knob("CLSKD_WGRAD_DEPTH", 0)
    print("total: " + "  ".join(f"{k} {v:.1f} us" for k, v in tot.items()))


if __name__ == "__main__":
    main()
