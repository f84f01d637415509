#!/bin/bash
# Iteration loop on one MI355X: GPU tests (optionally filtered by $1 = pytest -k expression),
# then the default bench line and a kernel trace of a short bench.  Each step time-limited.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/it
mkdir -p $O
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > $O/gt.log 2>&1
else
  timeout -k 10 500 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gt.log 2>&1
fi
timeout -k 10 200 python $R/bench.py --no-cpu-baseline > $O/b.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline > $O/tr.log 2>&1
echo ok
