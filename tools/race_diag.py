"""Locate a multi-stream replay mismatch: eager step vs StepExecutor (or StepGraph) replay on the
same batches, every tensor of the step's output tree compared (teacher / student forward
buffers, ReviewKD outputs, Gram slabs, loss slots); prints the differing leaves of each replay.

    python tools/race_diag.py [--replays 8] [--kind exec|graph] [--streams 4]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "speech-enhancement-clskd_amd"))

import torch  # noqa: E402

DEV = "cuda"


def leaves(x, name="", out=None, seen=None):
    from clskd import ops
    out = [] if out is None else out
    seen = set() if seen is None else seen
    if id(x) in seen:
        return out
    seen.add(id(x))
    if isinstance(x, torch.Tensor):
        out.append((name, x))
    elif isinstance(x, dict):
        for k in sorted(x, key=str):
            leaves(x[k], f"{name}.{k}", out, seen)
    elif isinstance(x, (list, tuple)):
        for i, v in enumerate(x):
            leaves(v, f"{name}[{i}]", out, seen)
    elif isinstance(x, ops.DeferredBN):
        leaves(x.raw, name + ".raw", out, seen)
        leaves(x.coef, name + ".coef", out, seen)
    elif isinstance(x, ops.GramSlabs):
        leaves(x.slabs, name + ".slabs", out, seen)
    elif hasattr(x, "owners"):
        leaves(x.owners, name + ".owners", out, seen)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replays", type=int, default=8)
    ap.add_argument("--kind", default="exec")
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--dump", action="store_true")
    ap.add_argument("--mutate", action="store_true",
                    help="scale a student weight in both models after two replays (re-capture)")
    args = ap.parse_args()
    from clskd.data import synthetic_pairs
    from clskd.graph import StepExecutor, StepGraph
    import test_gpu_parity as P
    batches = []
    for seed in (11, 12):
        n, c = synthetic_pairs(4, 32000, seed=seed)
        batches.append((torch.from_numpy(n).to(DEV), torch.from_numpy(c).to(DEV)))
    kd_e, kd_g = P._kd().set_precision("mixed"), P._kd().set_precision("mixed")
    g = StepExecutor(kd_g, *batches[0], nstreams=args.streams) if args.kind == "exec" else \
        StepGraph(kd_g, *batches[0])
    if args.kind == "exec" and args.dump:
        import ctypes as C
        from clskd import _lib
        L = _lib.load()
        n = L.clskd_exec_dump(g._ex, None, 0)
        b = C.create_string_buffer(int(n) + 1)
        L.clskd_exec_dump(g._ex, b, n + 1)
        print(b.value.decode(), flush=True)
    nbad = 0
    for r in range(args.replays):
        X, y = batches[r % 2]
        if args.mutate and r == 2:
            with torch.no_grad():
                for kd in (kd_e, kd_g):
                    kd.student.encoder[0][0].real_conv.weight.mul_(1.01)
        oe = kd_e.training_step((X, y), 0, return_parts=True)
        g(X, y)
        torch.cuda.synchronize()
        le = dict(leaves(oe))
        lg = leaves(g.out)
        bad = []
        for name, t in lg:
            e = le.get(name)
            if e is None or e.shape != t.shape or e.dtype != t.dtype:
                continue
            if not torch.equal(e, t):
                d = (e.double() - t.double()).abs()
                bad.append(f"{name} {tuple(t.shape)} max {float(d.max()):.3e} n {int((d > 0).sum())}")
        bad = [b for b in bad if not b.startswith((".s_enc[", ".s_dec["))]  # materialized once
        nbad += bool(bad)
        print(f"replay {r}: {len(lg)} leaves, {len(bad)} differ, captures {g.captures}", flush=True)
        for b in bad[:40]:
            print("   ", b, flush=True)
    print(f"{args.kind} streams={args.streams}: {nbad}/{args.replays} replays differ")


if __name__ == "__main__":
    main()
