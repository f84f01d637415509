#!/bin/bash
# Executor: host pacing (eager-like submission timing) and scheduling gates (student after the
# k-th teacher node), against eager.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/exgate
mkdir -p $O
run() {
  local name=$1; shift
  timeout -k 10 180 env "$@" > $O/$name.log 2>&1
  grep -o '"ms_per_step": [0-9.]*, "host_enqueue_ms_per_step": [0-9.]*' $O/$name.log | sed "s/^/$name /" >> $O/summary.txt
}
B="python $R/bench.py --no-cpu-baseline --steps 30 --warmup 5 --launch exec"
run own CLSKD_EXEC_OWN_STREAMS=1 $B
run pace15 CLSKD_EXEC_OWN_STREAMS=1 CLSKD_EXEC_PACE_NS=15000 $B
run pace25 CLSKD_EXEC_OWN_STREAMS=1 CLSKD_EXEC_PACE_NS=25000 $B
for k in 8 16 28 40; do
  run gate_s1_t$k CLSKD_EXEC_OWN_STREAMS=1 CLSKD_EXEC_GATE=$((100000 + 30000 + k)) $B
done
run eager python $R/bench.py --no-cpu-baseline --steps 30 --warmup 5 --launch eager
cat $O/summary.txt
