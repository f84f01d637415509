"""Per-kernel averages of every counter in the rocprofv3 --pmc CSVs under a directory
(run_counter_collection.csv files; kernels whose name contains 'conv_'), one line per
(pass directory, kernel).  Diagnostic.

    python tools/pmc_summary_kernels.py gpurun_out/pmchw
"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "")
            if "conv_" not in k:
                continue
            k = k.split("(")[0]
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[k].add(row.get("Dispatch_Id"))
        for k, cs in acc.items():
            n = max(1, len(disp[k]))
            vals = " ".join(f"{c}={v / n:.4g}" for c, v in sorted(cs.items()))
            print(f"{os.path.basename(os.path.dirname(f))} {k[:60]} n={n} {vals}")


if __name__ == "__main__":
    main()
