"""Per-kernel statistics of a rocprofv3 kernel trace split at bench.py's roctx ranges
(`clskd_census`: the census step on one stream; `clskd_timed`: exactly the K timed steps).

    rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d D -o run -- \
        python3 bench.py --steps K --warmup W --no-cpu-baseline
    python tools/region_stats.py D/run K out.json

The ranges are host-side push/pop pairs, each bracketed by a device synchronisation in bench.py,
so every kernel of the region starts and ends inside it.  Reports, per region: kernel launches,
summed kernel time (serialised view) and the union of busy intervals (device wall), per step for
the timed region, and every kernel instance's calls / average / total — the rocprof view of the
bench line's `avg_launch_us` (timed) and `isolated_avg_launch_us` (census)."""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import canonical  # noqa: E402


def _rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def ranges(marker_csv):
    """{name: [(start, end), ...]} of the roctx push/pop ranges."""
    out = collections.defaultdict(list)
    for r in _rows(marker_csv):
        name = None
        for key in ("Function", "Message", "Name", "Marker_Name"):
            v = r.get(key)
            if v and v.startswith("clskd_"):
                name = v
                break
        if name is None:
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e > s:
            out[name].append((s, e))
    return out


def union_ns(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def region(kernels, lo, hi, steps):
    sel = [k for k in kernels if k[1] >= lo and k[2] <= hi]
    per = collections.defaultdict(list)
    for name, s, e in sel:
        per[canonical(name)].append(e - s)
    tot = sum(e - s for _, s, e in sel)
    return dict(
        steps=steps, launches=len(sel), launches_per_step=round(len(sel) / steps, 2),
        kernel_ms_per_step=round(tot / steps / 1e6, 4),
        busy_union_ms_per_step=round(union_ns([(s, e) for _, s, e in sel]) / steps / 1e6, 4),
        kernels={k: dict(calls=len(v), calls_per_step=round(len(v) / steps, 2),
                         avg_us=round(sum(v) / len(v) / 1e3, 3), total_ms=round(sum(v) / 1e6, 4))
                 for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))})


def main():
    prefix, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    kernels = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
               for r in _rows(prefix + "_kernel_trace.csv")]
    rg = ranges(prefix + "_marker_api_trace.csv")
    res = {}
    for name, iv in rg.items():
        lo, hi = iv[-1]
        res[name] = region(kernels, lo, hi, steps if name == "clskd_timed" else 1)
    json.dump(res, open(out, "w"), indent=1)
    for name, r in res.items():
        top = list(r["kernels"].items())[:6]
        print(name, {k: v for k, v in r.items() if k != "kernels"})
        for k, v in top:
            print("   ", k, v)


if __name__ == "__main__":
    main()
