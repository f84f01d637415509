"""Timing-only modes of the halo-tiled fp32 conv (conv_halo32.hip) on the student's enc3 shape
(B=16, 32 -> 64 channels, 5x2 taps, stride-(2,1), Fo=16, T=643), against the fp32 engine.
Experiments build (CLSKD_LIB=exp).  Diagnostic.

    CLSKD_LIB=exp python tools/h32_modes.py [--one]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")]
import torch  # noqa: E402

from clskd import _lib, ops  # noqa: E402

DEV = "cuda"


def case(B, Fi, T, Cin, N, sf, taps):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, Fi, T, Cin, generator=g).to(DEV)
    Fo = (Fi - 1) // sf + 1 if sf == 2 else Fi
    w = torch.randn(N, len(taps), Cin, generator=g) * 0.05
    wp = ops.pack_weight(w.to(DEV), len(taps) * Cin)
    bias = torch.randn(N, generator=g).to(DEV)
    out = torch.empty(B, Fo, T, N, device=DEV)
    nblk = ops.conv_mblocks(B, Fo, T)
    st = torch.empty(nblk * N * 2, device=DEV, dtype=torch.float64)
    flops = 2.0 * B * Fo * T * N * len(taps) * Cin

    def run():
        ops.conv([ops.seg_bftc(x)], taps, B, Fo, T, N, wp, bias, out,
                 ops.OutMap(Fo * T * N, T * N, N), stride_f=sf, stats=st)
    return run, flops


def timeit(run, reps=20):
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    enc = [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)]
    if "--marks" in sys.argv:  # timeline of workgroup 0 (waves 0 and 4) on enc3
        import ctypes as C
        run, _ = case(16, 32, 643, 32, 64, 2, enc)
        _lib.set_knob("CLSKD_H32_DEBUG_MODE", 5)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        buf = (C.c_int64 * 128)()
        _lib.check(_lib.load().clskd_h32_marks(buf, 128), "marks")
        for w0 in (0, 64):
            m = [buf[w0 + i] for i in range(64)]
            n = next((i for i in range(1, 64) if m[i] <= 0 or m[i] < m[0]), 64)
            print(f"wave {w0 // 16}: " + " ".join(f"{(m[i] - m[i - 1]) * 0.01:.2f}" for i in range(1, n)))
        return
    if "--one" in sys.argv:  # the halo kernel on enc3 only (profiler runs)
        run, _ = case(16, 32, 643, 32, 64, 2, enc)
        for _ in range(10):
            run()
        torch.cuda.synchronize()
        return
    shapes = {"enc3 16x32x643 c32 n64": (16, 32, 643, 32, 64, 2, enc),
              "enc4 16x16x643 c64 n64": (16, 16, 643, 64, 64, 2, enc)}
    for name, sh in shapes.items():
        run, flops = case(*sh)
        for label, knobs in [("engine", {"CLSKD_NO_HALO32": 1}), ("halo", {}),
                             ("no DMA", {"CLSKD_H32_DEBUG_MODE": 1}),
                             ("reads once/chunk", {"CLSKD_H32_DEBUG_MODE": 2}),
                             ("no MFMA", {"CLSKD_H32_DEBUG_MODE": 3}),
                             ("no stores", {"CLSKD_H32_DEBUG_MODE": 4}),
                             ("no DMA, no stores", {"CLSKD_H32_DEBUG_MODE": 8}),
                             ("prologue only", {"CLSKD_H32_DEBUG_MODE": 9})]:
            prev = {k: _lib.set_knob(k, v) for k, v in knobs.items()}
            try:
                us = timeit(run)
                kn = ops.conv_kernel_of_last_launch()
            finally:
                for k, v in prev.items():
                    _lib.set_knob(k, v)
            print(f"{name:26s} {label:18s} {us:8.1f} us {flops / us / 1e6:7.1f} TF/s  {kn}")


if __name__ == "__main__":
    main()
