"""LSTM recurrence microbenchmark on the teacher (H=128) and student (H=32) C2 shapes."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")]
import torch  # noqa: E402

from clskd import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B, T = 16, 643
    for H in (128, 32):
        gx = torch.randn(2, 2 * B, T, 8 * H, device=dev) * 0.5
        whh = torch.randn(2, 4 * H, H, device=dev) * 0.05
        hs = torch.empty(2, 2 * B, T, H, device=dev)
        run = lambda: ops.lstm_recurrent(gx, 4 * H, T * 8 * H, 8 * H, whh, 2, 2 * B, T, H, hs,
                                         2 * B * T * H, T * H, H)
        for _ in range(2):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 10
        print(f"H={H:4d}: {us:8.1f} us per layer, {us / T * 1e3:7.1f} ns per step", flush=True)


if __name__ == "__main__":
    main()
