#!/bin/bash
# Eager vs hipGraph replay of the C2 step under the HIP runtime's graph-execution knobs
# (packet capture on/off, forced graph queue count).  One line per variant under gpurun_out/ge.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ge
mkdir -p $O
run() {  # name, env..., -- bench args
  local name=$1; shift
  echo "== $name" >> $O/summary.txt
  timeout -k 10 180 env "$@" > $O/$name.log 2>&1
  grep -o '"ms_per_step": [0-9.]*, "host_enqueue_ms_per_step": [0-9.]*' $O/$name.log >> $O/summary.txt || true
}
run eager python $R/bench.py --no-cpu-baseline --steps 20 --warmup 5
run graph python $R/bench.py --no-cpu-baseline --graph --steps 20 --warmup 5
run graph_q4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 python $R/bench.py --no-cpu-baseline --graph --steps 20 --warmup 5
run graph_nopc DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 python $R/bench.py --no-cpu-baseline --graph --steps 20 --warmup 5
run graph_nopc_q4 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 python $R/bench.py --no-cpu-baseline --graph --steps 20 --warmup 5
run eager2 python $R/bench.py --no-cpu-baseline --steps 20 --warmup 5
cat $O/summary.txt
