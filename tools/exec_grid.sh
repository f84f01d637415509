#!/bin/bash
# Executor vs eager under grid caps of the persistent conv kernels (CLSKD_G8_GRID / CLSKD_HALO_GRID).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/exgrid
mkdir -p $O
run() {
  local name=$1; shift
  timeout -k 10 180 env "$@" > $O/$name.log 2>&1
  grep -o '"ms_per_step": [0-9.]*, "host_enqueue_ms_per_step": [0-9.]*' $O/$name.log | sed "s/^/$name /" >> $O/summary.txt
}
B="python $R/bench.py --no-cpu-baseline --steps 30 --warmup 5"
run exec $B --launch exec
run eager $B --launch eager
for g in 192 128; do
  run exec_g$g CLSKD_G8_GRID=$g CLSKD_HALO_GRID=$g $B --launch exec
  run eager_g$g CLSKD_G8_GRID=$g CLSKD_HALO_GRID=$g $B --launch eager
done
run exec_own_g192 CLSKD_EXEC_OWN_STREAMS=1 CLSKD_G8_GRID=192 CLSKD_HALO_GRID=192 $B --launch exec
cat $O/summary.txt
