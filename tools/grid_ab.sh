#!/bin/bash
# C2 step with the persistent engines' grids capped (experiments library: CLSKD_G8_GRID /
# CLSKD_HALO_GRID), interleaved with the uncapped default; one box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-gridab}
mkdir -p $O
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for leg in d0:0:0 g224:224:0 g192:192:0 h224:0:224 d1:0:0 g240:240:0 g224b:224:0 d2:0:0; do
  IFS=: read name g h <<< "$leg"
  rc=0; CLSKD_LIB=exp CLSKD_G8_GRID=$g CLSKD_HALO_GRID=$h timeout -k 10 150 $B > $O/b_$name.log 2>&1 || rc=$?
  if [ $rc -ne 0 ]; then echo "stop $name rc=$rc"; exit $rc; fi
  echo "$name $(grep '^{' $O/b_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["host_enqueue_ms_per_step"], d["config"]["loss"])')"
done
