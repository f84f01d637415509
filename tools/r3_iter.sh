#!/bin/bash
# Round-3 iteration: executor + full-size mixed parity tests, C2 lines exec vs eager, C1 line.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v -s --timeout 600 --timeout-method thread -k "${1:-step_graph or c2_mixed or streaming_30s}" > $O/gt.log 2>&1
for v in exec eager exec eager; do
  timeout -k 10 180 python $R/bench.py --no-cpu-baseline --launch $v --steps 20 --warmup 5 > $O/b_$v.log 2>&1
  grep -o '"ms_per_step": [0-9.]*, "host_enqueue_ms_per_step": [0-9.]*' $O/b_$v.log | sed "s/^/$v /" >> $O/summary.txt
done
timeout -k 10 300 python $R/bench.py --c1 > $O/c1.log 2>&1
cat $O/summary.txt
