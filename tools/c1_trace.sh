#!/bin/bash
# C1 (B=1 eval forward) under a kernel trace: per-kernel durations and the gaps between them.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c1trace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --c1 --steps 10 --warmup 3 > $O/trace.log 2>&1
python3 - $O/trace/run_kernel_trace.csv <<'PY'
import csv, sys
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:70])
              for r in csv.DictReader(open(sys.argv[1])))
# the last forward: the final 66 kernels before the CPU legs
last = rows[-66:]
t0 = last[0][0]
busy = sum(e - s for s, e, _ in last)
span = last[-1][1] - t0
print(f"last 66 kernels: span {span/1e3:.1f} us, busy {busy/1e3:.1f} us, gaps {(span-busy)/1e3:.1f} us")
prev = t0
for s, e, n in last:
    print(f"{(s-prev)/1e3:7.2f} gap {(e-s)/1e3:7.2f} us  {n}")
    prev = e
PY
