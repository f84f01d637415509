#!/bin/bash
# C2 eager step under a kernel trace: per-stream busy time and kernel census of the timed steps.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c2trace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --launch ${1:-eager} > $O/trace.log 2>&1
python3 $R/tools/stream_busy.py $O/trace/run_kernel_trace.csv --steps 10 > $O/busy.txt
cat $O/busy.txt | head -70
