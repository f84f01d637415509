"""LSTM recurrence microbenchmark on the teacher (H=128) and student (H=32) C2 shapes, and the
student layer's backward (BPTT) with both kernels."""
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
    # backward (BPTT) of the student's layer: 2 weight sets x 2B sequences, single-wave kernel vs
    # the 4-wave k-sliced one (CLSKD_LSTM_BWD_WAVE 1 / 0)
    from clskd import _lib
    H = 32
    pre = torch.randn(2, 2 * B, T, 4 * H, device=dev) * 0.5
    dh = torch.randn(2, 2 * B, T, H, device=dev)
    whh = torch.randn(2, 4 * H, H, device=dev) * 0.05
    dg = torch.empty_like(pre)
    st = (2 * B * T * 4 * H, T * 4 * H, 4 * H)
    for wave in (0, 1, 0, 1):
        _lib.set_knob("CLSKD_LSTM_BWD_WAVE", wave)
        run = lambda: ops.lstm_bwd(pre, st, dh, (2 * B * T * H, T * H, H), whh, 2, 2 * B, T, H, dg, st)
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
        print(f"bwd H={H} wave={wave}: {us:8.1f} us per layer, {us / T * 1e3:7.1f} ns per step",
              flush=True)
    _lib.set_knob("CLSKD_LSTM_BWD_WAVE", 1)
    # the single-wave kernel with its gate-gradient reads issued together (CLSKD_LSTM_BWD_PIN)
    for pin in (0, 1, 0, 1):
        _lib.set_knob("CLSKD_LSTM_BWD_PIN", pin)
        run = lambda: ops.lstm_bwd(pre, st, dh, (2 * B * T * H, T * H, H), whh, 2, 2 * B, T, H, dg, st)
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
        print(f"bwd H={H} wave=1 pin={pin}: {us:8.1f} us per layer, {us / T * 1e3:7.1f} ns per step",
              flush=True)
    _lib.set_knob("CLSKD_LSTM_BWD_PIN", 1)


if __name__ == "__main__":
    main()
