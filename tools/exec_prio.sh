#!/bin/bash
# Executor stream priorities (own streams, capture-time tags: 1 student, 2 ReviewKD-enc, 3 teacher).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/exprio
mkdir -p $O
run() {
  local name=$1; shift
  timeout -k 10 180 env "$@" > $O/$name.log 2>&1
  grep -o '"ms_per_step": [0-9.]*, "host_enqueue_ms_per_step": [0-9.]*' $O/$name.log | sed "s/^/$name /" >> $O/summary.txt
}
B="python $R/bench.py --no-cpu-baseline --steps 30 --warmup 5 --launch exec"
run own CLSKD_EXEC_OWN_STREAMS=1 $B
run own_p8 CLSKD_EXEC_OWN_STREAMS=1 CLSKD_EXEC_PRIO=8 $B
run own_p2 CLSKD_EXEC_OWN_STREAMS=1 CLSKD_EXEC_PRIO=2 $B
run own_p4 CLSKD_EXEC_OWN_STREAMS=1 CLSKD_EXEC_PRIO=4 $B
run own_p6 CLSKD_EXEC_OWN_STREAMS=1 CLSKD_EXEC_PRIO=6 $B
run eager python $R/bench.py --no-cpu-baseline --steps 30 --warmup 5 --launch eager
cat $O/summary.txt
