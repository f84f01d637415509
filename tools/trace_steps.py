"""Steady-state per-step kernel table from a rocprofv3 kernel trace: kernels between the last
`n` step boundaries (the spkd_finalize launch ends each CLSKD step).  Diagnostic only.
    python tools/trace_steps.py run_kernel_trace.csv [n_steps] [top]"""
import collections
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_traffic import canonical  # noqa: E402


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    fin = [i for i, r in enumerate(rows) if "spkd_finalize" in r["Kernel_Name"]]
    sel = rows[fin[-n - 1] + 1: fin[-1] + 1]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in sel:
        k = canonical(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot = sum(v[1] for v in agg.values())
    print(f"{tot / n / 1e3:.3f} ms/step serialised kernel time, {len(sel) / n:.0f} launches/step")
    for k, (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{us / n:8.1f} us/step {c / n:5.1f} calls {us / c:7.1f} us avg  {k[:80]}")


if __name__ == "__main__":
    main()
