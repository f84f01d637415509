#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (serialised kernel times per step).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ts
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/log 2>&1
