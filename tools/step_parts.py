"""Critical-path probe of the C2 step: device time of the teacher forward alone, the student
side chain alone (student forward, ABF re-draw, ReviewKD fusions, MRSTFT), the Gram tail alone
and the full two-stream step, each averaged over `iters` eager iterations with HIP events.
Diagnostic only (rocprof's kernel trace serialises the two streams, so overlap is read here)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from clskd.data import synthetic_pairs  # noqa: E402


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    kd = bench.build_kd(dev, "step", "mixed")
    n, c = synthetic_pairs(bench.B_PER_GPU, bench.L, seed=1)
    X, y = torch.from_numpy(n).to(dev), torch.from_numpy(c).to(dev)
    spec = kd.teacher.spectrum(X)

    def teacher():
        kd.teacher.run(X, train=True, bn_updates=1, spec=spec, want_masks=False)

    def side():
        sf = kd.student.run(X, train=True, bn_updates=2, spec=spec, want_masks=False)
        kd._reinit_abf(None)
        kd.review_encoder.forward_bftc(sf["enc"])
        kd.review_decoder.forward_bftc([sf["dec_in"]] + sf["dec"][:5])
        buf = torch.empty(2, device=dev)
        kd.stft_loss(sf["out_wav"], y, out2=buf)

    def student():
        kd.student.run(X, train=True, bn_updates=2, spec=spec, want_masks=False)

    def full():
        kd.training_step((X, y))

    for name, fn in (("teacher forward", teacher), ("student forward", student),
                     ("side chain (student+ABF+MRSTFT)", side), ("full step (2 streams)", full)):
        print(f"{name:34s} {timeit(fn, iters):7.3f} ms", flush=True)


if __name__ == "__main__":
    main()
