#!/bin/bash
# teacher_ahead: parity test, then C2 eager with / without the overlap, back to back.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ahead
mkdir -p $O
rm -f $O/summary.txt
timeout -k 10 300 python -u -m pytest $R/tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "teacher_ahead or clskd_step_golden" > $O/gt.log 2>&1
for v in ahead no ahead no; do
  extra=""; [ $v = no ] && extra="--no-ahead"
  timeout -k 10 180 python $R/bench.py --no-cpu-baseline --launch eager --steps 20 --warmup 5 $extra > $O/b_$v.log 2>&1
  grep -o '"ms_per_step": [0-9.]*, "host_enqueue_ms_per_step": [0-9.]*' $O/b_$v.log | sed "s/^/$v /" >> $O/summary.txt
done
cat $O/summary.txt
