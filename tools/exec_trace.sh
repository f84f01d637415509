#!/bin/bash
# Kernel traces (queue / stream ids, start / end) of the C2 step: eager vs executor launch.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/extr
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in eager exec; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o run -- python3 $R/bench.py --no-cpu-baseline --launch $v --steps 6 --warmup 3 > $O/$v.log 2>&1
done
echo ok
