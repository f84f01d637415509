"""Per-step kernel time table from a rocprofv3 *_kernel_stats.csv (steps = warmup + timed)."""
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_traffic import canonical  # noqa: E402


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total {tot / steps / 1e6:.3f} ms/step over {steps} steps")
    for r in rows[: int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
        print(f"{float(r['TotalDurationNs']) / steps / 1e3:8.1f} us/step {int(r['Calls']) / steps:6.1f} "
              f"calls {float(r['AverageNs']) / 1e3:7.1f} us avg  {canonical(r['Name'])[:80]}")


if __name__ == "__main__":
    main()
