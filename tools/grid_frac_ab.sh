#!/bin/bash
# C2 step: conv_gemm8 concurrent-step grid fraction sweep (CLSKD_STEP_G8_GRID_FRAC), interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-gridfrac}
mkdir -p $O
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for leg in a:0.875 b:0.8125 c:0.75 d:0.875 e:0.8125 f:0.6875 g:0.875; do
  name=${leg%%:*}; fr=${leg#*:}
  rc=0; CLSKD_STEP_G8_GRID_FRAC=$fr timeout -k 10 150 $B > $O/b_$name.log 2>&1 || rc=$?
  if [ $rc -ne 0 ]; then echo "stop $name rc=$rc"; exit $rc; fi
  echo "$name $fr $(grep '^{' $O/b_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["host_enqueue_ms_per_step"])')"
done
