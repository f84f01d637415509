"""Per-call census of the C3 backward's GEMM launches: every `ops.conv_wgrad` (weight gradient)
and `ops.conv` (data gradient / forward) call of one eager training step, each bracketed by
device synchronisation and HIP events (a sleep kernel ahead of the first event hides the host
launch latency), grouped by shape, call site and dispatched kernel.  Diagnostic only (serialises the step).

    python tools/bwd_census.py [--precision mixed] [--top 40]
"""
import argparse
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="mixed")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--batch", type=int, default=16)
    args = ap.parse_args()
    import bench
    from clskd import config as cfg
    from clskd import ops
    from clskd.data import synthetic_pairs
    from clskd.train import FlatAdam, FlatParams
    dev = torch.device("cuda", 0)
    kd = bench.build_kd(dev, "step", args.precision)
    flat = FlatParams(kd.student)
    opt = FlatAdam(flat, lr=cfg.learning_rate)
    noisy, clean = synthetic_pairs(args.batch, 64000, seed=1)
    X, y = torch.from_numpy(noisy).to(dev), torch.from_numpy(clean).to(dev)
    for _ in range(3):
        kd.train_step((X, y), flat, opt)
    torch.cuda.synchronize()

    rec = collections.defaultdict(list)

    def wrap(name, fn, keyf):
        def w(*a, **k):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s = torch.cuda.current_stream()
            # keep the device busy while the host enqueues the call, so the event pair spans
            # device time only (not the Python launch latency of a short launch)
            torch.cuda._sleep(2_000_000)
            e0.record(s)
            r = fn(*a, **k)
            e1.record(s)
            torch.cuda.synchronize()
            f = sys._getframe(1)
            site = f"{os.path.basename(f.f_code.co_filename)}:{f.f_lineno}"
            kern = ops.conv_kernel_of_last_launch() if name == "conv" else ""
            rec[(name,) + keyf(a, k) + (site, str(kern)[:60])].append(e0.elapsed_time(e1) * 1e3)
            return r
        return w

    def ckey(a, k):
        segs, taps, B, Fo, To, N = a[:6]
        cin = sum(int(sg.tensor.shape[-1]) if hasattr(sg, "tensor") else 0 for sg in segs)
        dt = str(getattr(segs[0], "tensor", torch.empty(0)).dtype).replace("torch.", "")
        return (f"M={B * Fo * To}", f"N={N}", f"K={len(taps) * cin}", f"taps={len(taps)}",
                f"nseg={len(segs)}", dt)

    orig = ops.conv_wgrad, ops.conv
    ops.conv_wgrad = wrap("wgrad", orig[0], ckey)
    ops.conv = wrap("conv", orig[1], ckey)
    try:
        kd.train_step((X, y), flat, opt)
    finally:
        ops.conv_wgrad, ops.conv = orig
    torch.cuda.synchronize()
    tot = collections.Counter()
    rows = []
    for key, v in rec.items():
        tot[key[0]] += sum(v)
        m, n, kk = (int(key[i].split("=")[1]) for i in (1, 2, 3))
        fl = 2.0 * m * n * kk * len(v)
        rows.append((sum(v), key, len(v), fl / (sum(v) * 1e-6) / 1e12))
    rows.sort(reverse=True)
    for us, key, cnt, tf in rows[:args.top]:
        print(f"{us:9.1f} us  x{cnt:<3d} {tf:7.1f} TF/s  {' '.join(key)}")
    for k, v in tot.items():
        print(f"total {k}: {v / 1e3:.3f} ms over {sum(len(x) for kk, x in rec.items() if kk[0] == k)} calls")


if __name__ == "__main__":
    main()
