"""Run one chain of the C2 step alone (student forward | ReviewKD decoder | ReviewKD encoder |
teacher forward), `iters` times after 2 warm-ups — for a rocprofv3 kernel trace of that chain's
kernels in isolation.  Diagnostic only.

    rocprofv3 --kernel-trace --stats -d DIR -o run -- python3 tools/chain_profile.py student 3
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from clskd.data import synthetic_pairs  # noqa: E402


def main():
    which = sys.argv[1]
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    kd = bench.build_kd(dev, "step", "mixed")
    n, c = synthetic_pairs(bench.B_PER_GPU, bench.L, seed=1)
    X = torch.from_numpy(n).to(dev)
    spec = kd.teacher.spectrum(X)
    sf = kd.student.run(X, train=True, bn_updates=2, spec=spec, want_masks=False)
    fns = {
        "student": lambda: kd.student.run(X, train=True, bn_updates=2, spec=spec, want_masks=False),
        "rdec": lambda: kd.review_decoder.forward_bftc([sf["dec_in"]] + sf["dec"][:5]),
        "renc": lambda: kd.review_encoder.forward_bftc(sf["enc"]),
        "teacher": lambda: kd.teacher.run(X, train=True, bn_updates=1, spec=spec, want_masks=False),
    }
    fn = fns[which]
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{which}: {e0.elapsed_time(e1) / iters:.3f} ms per run")


if __name__ == "__main__":
    main()
