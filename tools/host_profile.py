"""Host-side profile of the C3 training step (cProfile over K steps after warm-up) — where the
host spends its enqueue time.  Diagnostic only.
    python tools/host_profile.py [steps] [top]"""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "speech-enhancement-clskd_amd"))


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    mode = os.environ.get("MODE", "train")
    import bench
    from clskd.data import synthetic_pairs
    from clskd.train import FlatAdam, FlatParams
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    kd = bench.build_kd(dev, "step", "mixed")
    Xs, Ys = [], []
    for k in range(bench.NBATCH):
        noisy, clean = synthetic_pairs(bench.B_PER_GPU, bench.L, seed=1000 + k)
        Xs.append(torch.from_numpy(noisy).to(dev))
        Ys.append(torch.from_numpy(clean).to(dev))
    flat = FlatParams(kd.student)
    opt = FlatAdam(flat, lr=6e-4)
    if mode == "train":
        step = lambda i: kd.train_step((Xs[i % len(Xs)], Ys[i % len(Ys)]), flat, opt)
    else:
        def step(i):
            with torch.no_grad():
                return kd.training_step((Xs[i % len(Xs)], Ys[i % len(Ys)]), i)
    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(top)


if __name__ == "__main__":
    main()
