#!/bin/bash
# C2 step: executor with / without capture-time stream tags, on the step's side streams or its own, vs eager.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/exab
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "step_graph" > $O/gt.log 2>&1
run() {
  local name=$1; shift
  timeout -k 10 180 env "$@" > $O/$name.log 2>&1
  grep -o '"ms_per_step": [0-9.]*, "host_enqueue_ms_per_step": [0-9.]*' $O/$name.log | sed "s/^/$name /" >> $O/summary.txt
}
for i in 1; do
  run exec_tags python $R/bench.py --no-cpu-baseline --launch exec --steps 30 --warmup 5
  run exec_tags_own CLSKD_EXEC_OWN_STREAMS=1 python $R/bench.py --no-cpu-baseline --launch exec --steps 30 --warmup 5
  run exec_notags_own CLSKD_EXEC_TAGS=0 CLSKD_EXEC_OWN_STREAMS=1 python $R/bench.py --no-cpu-baseline --launch exec --steps 30 --warmup 5
  run eager python $R/bench.py --no-cpu-baseline --launch eager --steps 30 --warmup 5
  run exec_q8 GPU_MAX_HW_QUEUES=8 python $R/bench.py --no-cpu-baseline --launch exec --steps 30 --warmup 5
  run eager_q8 GPU_MAX_HW_QUEUES=8 python $R/bench.py --no-cpu-baseline --launch eager --steps 30 --warmup 5
  run exec_tags python $R/bench.py --no-cpu-baseline --launch exec --steps 30 --warmup 5
  run eager python $R/bench.py --no-cpu-baseline --launch eager --steps 30 --warmup 5
done
cat $O/summary.txt
