"""Concurrency timeline of the last steps in a rocprofv3 kernel trace of bench.py: per stream,
busy time and the time the stream's last kernel of the step ends; the step's intervals by
number of concurrently running kernels (where only one small kernel runs, the chip idles).
Diagnostic only.    python tools/step_timeline.py run_kernel_trace.csv [n_steps]"""
import collections
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_traffic import canonical  # noqa: E402


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    fin = [i for i, r in enumerate(rows) if "spkd_finalize" in r["Kernel_Name"]]
    for s in range(n):
        sel = rows[fin[-n - 1 + s] + 1: fin[-n + s] + 1]
        t0 = int(fin and rows[fin[-n - 1 + s]]["End_Timestamp"])
        t1 = max(int(r["End_Timestamp"]) for r in sel)
        print(f"step {s}: {(t1 - t0) / 1e3:.1f} us from previous finalize end, {len(sel)} kernels")
        per = collections.defaultdict(lambda: [0, 0, 1 << 62, 0])
        for r in sel:
            k = r["Queue_Id"]
            a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            per[k][0] += b - a
            per[k][1] += 1
            per[k][2] = min(per[k][2], a)
            per[k][3] = max(per[k][3], b)
        for k, (busy, cnt, a, b) in sorted(per.items(), key=lambda kv: kv[1][2]):
            print(f"  queue {k:>4}: {cnt:4d} kernels, busy {busy / 1e3:7.1f} us, "
                  f"first start +{(a - t0) / 1e3:7.1f}, last end +{(b - t0) / 1e3:7.1f}")
        # concurrency histogram: sweep start/end events, attributing single-kernel spans
        ev = sorted([(int(r["Start_Timestamp"]), 1, i) for i, r in enumerate(sel)] +
                    [(int(r["End_Timestamp"]), -1, i) for i, r in enumerate(sel)],
                    key=lambda e: (e[0], e[1]))
        hist = collections.Counter()
        solo = collections.Counter()
        running, last = set(), t0
        for t, d, i in ev:
            if t > last:
                hist[len(running)] += t - last
                if len(running) == 1:
                    solo[canonical(sel[next(iter(running))]["Kernel_Name"])] += t - last
                last = t
            if d > 0:
                running.add(i)
            else:
                running.discard(i)
        print("  time by concurrent kernels: " +
              ", ".join(f"{c}: {v / 1e3:.0f} us" for c, v in sorted(hist.items())))
        print("  running alone (top): " + ", ".join(f"{k[:40]} {v / 1e3:.0f}" for k, v in solo.most_common(8)))


if __name__ == "__main__":
    main()
