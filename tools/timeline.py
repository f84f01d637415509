"""Per-queue timeline of one step from a rocprofv3 kernel trace (csv): busy time, span and the
kernels in order with gaps.  Diagnostic only.  usage: timeline.py run_kernel_trace.csv [--full]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # step boundary marker: the spkd finalize kernel (one per step)
    fin = [i for i, r in enumerate(rows) if "spkd_finalize" in r["Kernel_Name"]]
    a, b = fin[-3] + 1, fin[-2] + 1
    step = rows[a:b]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in step)
    print(f"step span {(t1 - t0) / 1e3:.1f} us, {len(step)} kernels")
    byq = collections.defaultdict(list)
    for r in step:
        byq[r["Queue_Id"]].append(r)
    agg = collections.defaultdict(lambda: [0, 0.0])
    for q, rs in byq.items():
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs)
        print(f"queue {q}: {len(rs)} kernels, busy {busy / 1e3:.1f} us, "
              f"first {(int(rs[0]['Start_Timestamp']) - t0) / 1e3:.1f} last end "
              f"{(int(rs[-1]['End_Timestamp']) - t0) / 1e3:.1f}")
    for r in step:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
        agg[n][0] += 1
        agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print("\nper kernel (both queues):")
    for n, (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"{us:9.1f} us {c:4d}x  {n}")
    if "--full" in sys.argv:
        for q, rs in byq.items():
            print("=== queue", q)
            prev = None
            for r in rs:
                s = (int(r["Start_Timestamp"]) - t0) / 1e3
                e = (int(r["End_Timestamp"]) - t0) / 1e3
                gap = s - prev if prev is not None else 0.0
                prev = e
                print(f"{s:9.1f} {e - s:8.1f} gap{gap:7.1f}  {r['Kernel_Name'].split('(')[0][:70]}")


if __name__ == "__main__":
    main()
