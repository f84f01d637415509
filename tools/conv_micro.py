"""Single-layer conv-engine microbenchmark on the teacher's bf16 shapes (C2 workload, B=16,
T=643): encoder 5x2 stride-(2,1) layers, a decoder polyphase parity-0 layer and a ReviewKD 3x3.
Times `iters` back-to-back launches with HIP events.  Diagnostic only.

    python tools/conv_micro.py [--iters 50] [--only enc4,dec1]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")]
import torch  # noqa: E402

from clskd import ops  # noqa: E402

B, T = 16, 643
ENC = [(2, 32, 256), (32, 64, 128), (64, 128, 64), (128, 256, 32), (256, 256, 16), (256, 256, 8)]
CFGS = {f"enc{i}": ("enc", ci, co, fi) for i, (ci, co, fi) in enumerate(ENC) if ci >= 8}
CFGS.update({
    "dec1": ("dec", 512, 256, 8),     # 6 taps x 512 -> K 3072
    "dec3": ("dec", 256, 128, 32),
    "dec5": ("dec", 64, 32, 128),
    "abf3": ("abf", 64, 256, 16),     # 3x3, 64 -> 256
    "abf4": ("abf", 64, 128, 32),     # 3x3, 64 -> 128 (the 256x128-tile engine config)
    "abf5": ("abf", 64, 64, 64),
    # plain GEMMs through the same engine (1x1 "conv", contiguous rows: no tap gather)
    "pw_enc4": ("pw", 2560, 256, 8),          # enc4's M x N x K without the im2col gather
    "pw64k": ("pw", 4096, 256, 1, 16, 4096),  # M 65536 x N 256 x K 4096: 256 tiles, 64 K-tiles each
})


def make(kind, ci, co, fi, B=B, T=T, dev=None):
    g = torch.Generator(device="cpu").manual_seed(0)
    x = (torch.randn(B, fi, T, ci, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    if kind == "pw":
        taps = [(0, 0)]
        Fo, To, sf, omap_f = fi, T, 1, 1
    elif kind == "enc":
        taps = [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)]
        Fo, To, sf, omap_f = fi // 2, T, 2, 1
    elif kind == "dec":
        taps = [(dF, -kt) for dF in (1, 0, -1) for kt in (0, 1)]
        Fo, To, sf, omap_f = fi, T, 1, 2
    else:
        taps = [(kf - 1, kt - 1) for kf in range(3) for kt in range(3)]
        Fo, To, sf, omap_f = fi, T, 1, 1
    K = len(taps) * ci
    w = (torch.randn(co, K, generator=g) * 0.05).to(dev)
    wp = ops.pack_weight(w.view(co, len(taps), ci), K, "bf16")
    bias = torch.zeros(co, device=dev)
    out = torch.empty(B, Fo * omap_f, To, co, device=dev, dtype=torch.bfloat16)
    omap = ops.OutMap(Fo * omap_f * To * co, To * co, co, of_mul=omap_f, of_add=0)
    nblk = ops.conv_mblocks(B, Fo, To)
    st = torch.empty(nblk * co * 2, device=dev, dtype=torch.float64)
    seg = ops.seg_bftc(x)

    def run():
        ops.conv([seg], taps, B, Fo, To, co, wp, bias, out, omap, stride_f=sf, stats=st)
    run.out = out
    return run, 2.0 * B * Fo * To * co * K, (B * Fo * To, co, K)


def ab(a, dev, names):
    """--ab KNOB=v1,v2: the knob's values interleaved over --rounds rounds in this one process
    (cdna_hip_programming.md §5.4 rule 24); median and min per value."""
    from clskd import _lib
    knob, vals = a.ab.split("=")
    vals = [int(v) for v in vals.split(",")]
    for name in names:
        run, fl, (M, N, K) = make(*CFGS[name], dev=dev)
        res = {v: [] for v in vals}
        for r in range(a.rounds):
            for v in vals:
                _lib.set_knob(knob, v)
                for _ in range(2):
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) * 1e3 / a.iters)
        line = " ".join(f"{knob}={v}: med {sorted(t)[len(t) // 2]:7.1f} min {min(t):7.1f} us "
                        f"({fl / min(t) / 1e6:6.1f} TF/s)" for v, t in res.items())
        print(f"{name:8s} M={M:7d} N={N:4d} K={K:5d}  {line}  [{ops.conv_kernel_of_last_launch()}]",
              flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", default="")
    ap.add_argument("--ab", default="", help="KNOB=v1,v2: interleaved A/B of a dispatch knob")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    names = [n for n in CFGS if not a.only or n in a.only.split(",")]
    if a.ab:
        return ab(a, dev, names)
    for name in names:
        run, fl, (M, N, K) = make(*CFGS[name], dev=dev)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        print(f"{name:6s} M={M:7d} N={N:4d} K={K:5d}  {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
