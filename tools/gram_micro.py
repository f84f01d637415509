"""Isolated timing of clskd_gram_partial on step-like views (HIP events, 20 reps): bf16 and fp32
feature maps [B, P, C] channels-last, with and without the folded BatchNorm affine.  Prints
GB/s of algorithmic input bytes.  Diagnostic only.
    python tools/gram_micro.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "speech-enhancement-clskd_amd"))
from clskd import ops  # noqa: E402

CASES = [  # (name, B, P, C, dtype, affine)
    ("t_enc_bf16_c128", 16, 161 * 643 // 2, 128, torch.bfloat16, False),
    ("t_enc_bf16_c256", 16, 41 * 643, 256, torch.bfloat16, True),
    ("s_enc_f32_c32", 16, 81 * 643, 32, torch.float32, False),
    ("s_enc_f32_c64", 16, 41 * 643, 64, torch.float32, True),
]


CHUNKS = [int(c) for c in os.environ.get("CHUNKS", "16384 8192 4096 2048").split()]


def main():
    dev = torch.device("cuda:0")
    for name, B, P, C, dt, aff in CASES:
        x = torch.randn(B, P, C, device=dev).to(dt)
        coef = None
        if aff:
            coef = torch.cat([torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)]).float()
        v = ops.GramView(x, 0, P * C, P, C, 0, C, coef)
        for ch in CHUNKS:
            for _ in range(3):
                ops.GramSlabs([v], B, ch)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            e0.record()
            for _ in range(reps):
                ops.GramSlabs([v], B, ch)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            nbytes = x.numel() * x.element_size()
            nsl = -(-P // max(1, ch // C))
            print(f"{name:18s} chunk {ch:6d} ({nsl:5d} slabs) {nbytes / 1e6:8.1f} MB {us:8.1f} us "
                  f"{nbytes / us / 1e6:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
