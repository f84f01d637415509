"""Mean PMC counter values per dispatch of kernels matching a substring, from rocprofv3
run_counter_collection.csv files (one per pass).

    python tools/pmc_summary.py <substring> pass1.csv [pass2.csv ...]
"""
import collections
import csv
import sys


def main():
    key = sys.argv[1]
    vals = collections.defaultdict(list)
    dur = []
    for path in sys.argv[2:]:
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(path)):
            if key not in r["Kernel_Name"]:
                continue
            per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
            if path == sys.argv[2]:
                per[r["Dispatch_Id"]]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for dct in per.values():
            for k, v in dct.items():
                vals[k].append(v)
    for k in sorted(vals):
        v = vals[k]
        print(f"{k:34s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
