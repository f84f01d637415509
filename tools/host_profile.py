"""Where the eager C2 step's host enqueue time goes: cProfile over K eager steps of the bench
workload (B=16 x 4 s, precision='mixed', ABF re-draw per step), no synchronisation inside the
profiled loop (the device runs behind; the host only enqueues).  Prints the host ms per step and
the top functions by own time and by cumulative time.

    python tools/host_profile.py [--steps 20] [--top 40]
"""
import argparse
import cProfile
import gc
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "speech-enhancement-clskd_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    import bench
    from clskd import config as cfg  # noqa: F401
    from clskd.data import synthetic_pairs
    dev = torch.device("cuda", 0)
    kd = bench.build_kd(dev, "step", "mixed")
    noisy, clean = synthetic_pairs(16, 64000, seed=1)
    X, y = torch.from_numpy(noisy).to(dev), torch.from_numpy(clean).to(dev)
    with torch.no_grad():
        for i in range(4):
            kd.training_step((X, y), i)
    torch.cuda.synchronize()
    gc.collect()
    gc.freeze()
    t0 = time.perf_counter()
    with torch.no_grad():
        for i in range(args.steps):
            kd.training_step((X, y), i)
    plain = (time.perf_counter() - t0) / args.steps * 1e3
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    with torch.no_grad():
        pr.enable()
        for i in range(args.steps):
            kd.training_step((X, y), i)
        pr.disable()
    torch.cuda.synchronize()
    print(f"host enqueue {plain:.3f} ms/step without the profiler")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(args.top)
    st.sort_stats("cumulative").print_stats(args.top)


if __name__ == "__main__":
    main()
