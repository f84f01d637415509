"""Phase breakdown of one fused streaming hop (clskd_stream_hop, stream 0) from the in-kernel
wall-clock marks of the -DCLSKD_EXPERIMENTS library (diagnostic; CLSKD_LIB=exp is set here).

    python tools/hop_marks.py [--streams B] [--hops N]
"""
import argparse
import ctypes as C
import os
import sys

os.environ["CLSKD_LIB"] = "exp"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from clskd import _lib, ops  # noqa: E402
from clskd import config as cfg  # noqa: E402
from clskd.data import synthetic_pairs  # noqa: E402
from clskd.model import DCCRN  # noqa: E402
from clskd.streaming import HOP, FusedStreamingDCCRN  # noqa: E402
from clskd.weights import STUDENT_SEED, apply_recipe  # noqa: E402

NAMES = ["stft", "enc0", "enc1", "enc2", "enc3", "enc4", "enc5", "lstm0", "lstm1", "proj",
         "dec0", "dec1", "dec2", "dec3", "dec4", "dec5", "mask", "istft", "ola"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=1)
    ap.add_argument("--hops", type=int, default=200)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT), STUDENT_SEED).to(dev).eval()
    noisy, _ = synthetic_pairs(a.streams, a.hops * HOP, seed=3)
    x = torch.from_numpy(noisy).to(dev)
    s = FusedStreamingDCCRN(m, a.streams)
    lib = ops.lib()
    acc = [0.0] * len(NAMES)
    n = 0
    buf = (C.c_int64 * 40)()
    inner = [0.0] * 6
    clk = [0.0, 0.0]
    for t in range(a.hops):
        s.step(x[:, t * HOP:(t + 1) * HOP])
        if t >= 20:
            torch.cuda.synchronize()
            _lib.check(lib.clskd_stream_hop_marks(buf, 40), "marks")
            for i in range(len(NAMES)):
                acc[i] += (buf[i + 1] - buf[i]) * 10e-3  # 100 MHz ticks -> us
            clk[0] += (buf[39] - buf[38]) / ((buf[19] - buf[0]) * 10e-9) / 1e9  # GHz
            clk[1] += buf[30] - buf[38]  # cycles of one global load round trip (+ a few)
            # inside conv (enc0, enc4, dec1): K loop done, partials barrier
            for k, (st, m) in enumerate([(1, 32), (5, 34), (11, 36)]):
                inner[2 * k] += (buf[m] - buf[st]) * 10e-3
                inner[2 * k + 1] += (buf[m + 1] - buf[m]) * 10e-3
            n += 1
    tot = sum(acc) / n
    print(f"fused hop, {a.streams} streams, mean over {n} hops: {tot:.1f} us (stream 0, kernel start -> end)")
    for name, v in zip(NAMES, acc):
        print(f"  {name:6s} {v / n:7.2f} us  {100 * v / n / tot:5.1f} %")
    print(f"shader clock {clk[0] / n:.2f} GHz; one dependent global load {clk[1] / n:.0f} cycles")
    for k, name in enumerate(["enc0", "enc4", "dec1"]):
        print(f"  {name}: previous phase end -> K loop done {inner[2 * k] / n:6.2f} us, partials + barrier {inner[2 * k + 1] / n:6.2f} us")


if __name__ == "__main__":
    main()
