"""Per-stream busy time of the last N steps of a rocprofv3 kernel trace (C2 bench) and the kernel
census by stream: which stream's chain sets the step.  Diagnostic.

    python tools/stream_busy.py run_kernel_trace.csv --steps 10
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--per-step", type=int, default=0, help="launches per step (0: infer from the SPKD finalize)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id", r["Queue_Id"]),
                 r["Kernel_Name"].split("(")[0][:80]) for r in rows)
    per = a.per_step
    if not per:
        # the bench's timed region is the tail: take the last steps by count of a once-per-step kernel
        marks = [i for i, e in enumerate(ev) if "ola_kernel" in e[3]]
        per = (marks[-1] - marks[-1 - a.steps]) // a.steps if len(marks) > a.steps else len(ev) // 20
    win = ev[-per * a.steps:]
    t0, t1 = win[0][0], max(e[1] for e in win)
    span = (t1 - t0) / 1e3 / a.steps
    print(f"{len(win)} kernels in the last {a.steps} steps ({per}/step); span {span:.1f} us/step")
    busy = collections.defaultdict(int)
    cnt = collections.Counter()
    ker = collections.defaultdict(lambda: collections.defaultdict(float))
    for s, e, q, n in win:
        busy[q] += e - s
        cnt[q] += 1
        ker[q][n] += (e - s) / 1e3 / a.steps
    for q in sorted(busy, key=lambda k: -busy[k]):
        print(f"stream {q}: {busy[q] / 1e3 / a.steps:8.1f} us/step busy, {cnt[q] / a.steps:5.1f} launches/step")
        for n, v in sorted(ker[q].items(), key=lambda kv: -kv[1])[:12]:
            print(f"     {v:8.1f}  {n}")


if __name__ == "__main__":
    main()
