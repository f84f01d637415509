#!/bin/bash
# Step-executor iteration: executor parity tests, then C2 lines eager vs exec (two each).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ex
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${1:-step_graph}" > $O/gt.log 2>&1
for v in exec eager exec eager; do
  timeout -k 10 180 python $R/bench.py --no-cpu-baseline --launch $v --steps 20 --warmup 5 > $O/b_$v.log 2>&1
  grep -o '"ms_per_step": [0-9.]*, "host_enqueue_ms_per_step": [0-9.]*' $O/b_$v.log | sed "s/^/$v /" >> $O/summary.txt
done
cat $O/summary.txt
