#!/bin/bash
# Serial A/B: the step on ONE stream, eager vs executor replay (separates schedule effects from
# kernel / memory-layout effects of the captured step).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/exser
mkdir -p $O
run() {
  local name=$1; shift
  timeout -k 10 180 env "$@" > $O/$name.log 2>&1
  grep -o '"ms_per_step": [0-9.]*, "host_enqueue_ms_per_step": [0-9.]*' $O/$name.log | sed "s/^/$name /" >> $O/summary.txt
}
B="python $R/bench.py --no-cpu-baseline --steps 30 --warmup 5"
run eager_serial CLSKD_SERIAL_STREAMS=1 $B --launch eager
run exec_serial CLSKD_EXEC_STREAMS=1 $B --launch exec
run exec_serial_capture CLSKD_SERIAL_STREAMS=1 $B --launch exec
run graph_serial CLSKD_SERIAL_STREAMS=1 $B --launch graph
run eager $B --launch eager
run exec $B --launch exec
cat $O/summary.txt
