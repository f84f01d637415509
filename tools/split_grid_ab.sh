#!/bin/bash
# C2 step: conv_split3 (student fp32 layers, split products) grid capped (experiments library,
# CLSKD_SPLIT_GRID = CUs spanned), interleaved with the uncapped default.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-splitgrid}
mkdir -p $O
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for leg in a:0 b:224 c:192 d:0 e:224 f:160 g:0; do
  name=${leg%%:*}; g=${leg#*:}
  rc=0; CLSKD_LIB=exp CLSKD_SPLIT_GRID=$g timeout -k 10 150 $B > $O/b_$name.log 2>&1 || rc=$?
  if [ $rc -ne 0 ]; then echo "stop $name rc=$rc"; exit $rc; fi
  echo "$name $g $(grep '^{' $O/b_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["host_enqueue_ms_per_step"])')"
done
