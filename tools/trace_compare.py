"""Compare two rocprofv3 kernel traces of the C2 bench (e.g. eager vs executor launch): per-queue
kernel counts, the timed steps' wall span, average concurrency, and per-kernel mean durations.
Diagnostic only.

    python tools/trace_compare.py A/run_kernel_trace.csv B/run_kernel_trace.csv [--last N]
"""
import argparse
import collections
import csv


def load(path, last):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Stream_Id"],
                 r["Kernel_Name"]) for r in rows)
    ev = ev[-last:] if last else ev
    return ev


def summary(ev, label):
    t0, t1 = ev[0][0], max(e[1] for e in ev)
    busy = sum(e[1] - e[0] for e in ev)
    q = collections.Counter((e[2], e[3]) for e in ev)
    # time with >= k kernels running
    pts = sorted([(e[0], 1) for e in ev] + [(e[1], -1) for e in ev])
    cur, last_t, hist = 0, pts[0][0], collections.Counter()
    for t, d in pts:
        hist[cur] += t - last_t
        cur += d
        last_t = t
    span = t1 - t0
    print(f"== {label}: {len(ev)} kernels, span {span / 1e6:.3f} ms, summed {busy / 1e6:.3f} ms, "
          f"avg concurrency {busy / span:.2f}")
    print("   queues (queue, stream): kernels", dict(q.most_common()))
    print("   time at concurrency k:", {k: round(v / span, 3) for k, v in sorted(hist.items())})
    per = collections.defaultdict(list)
    for s, e, _, _, n in ev:
        per[n.split("(")[0][:70]].append((e - s) / 1e3)
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--last", type=int, default=209 * 4)
    a = ap.parse_args()
    pa = summary(load(a.a, a.last), a.a)
    pb = summary(load(a.b, a.last), a.b)
    rows = []
    for k in set(pa) | set(pb):
        ma = sum(pa.get(k, [0])) / max(1, len(pa.get(k, [])))
        mb = sum(pb.get(k, [0])) / max(1, len(pb.get(k, [])))
        rows.append((sum(pb.get(k, [])) - sum(pa.get(k, [])), k, len(pa.get(k, [])), ma, len(pb.get(k, [])), mb))
    rows.sort(reverse=True)
    print("kernel (total delta us over the window; count / mean us in A, B):")
    for d, k, na, ma, nb, mb in rows[:25]:
        print(f"  {d:9.1f}  {k:70s} {na:4d} {ma:8.1f} | {nb:4d} {mb:8.1f}")


if __name__ == "__main__":
    main()
