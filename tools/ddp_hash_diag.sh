#!/bin/bash
# C3 parameter hashes after the bench's steps: executor vs eager, one rank and two (gloo, one GPU)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-ddpdiag}
mkdir -p $O
for g in 1 2; do
  for l in exec eager; do
    rc=0; CLSKD_DIST_BACKEND=gloo CLSKD_BENCH_DEVICE=0 timeout -k 10 300 python $R/bench.py --gpus $g --train --abf-reinit once --launch $l --steps 2 --warmup 1 $EXTRA > $O/g${g}_$l.log 2>&1 || rc=$?
    if [ $rc -ne 0 ]; then tail -20 $O/g${g}_$l.log; exit $rc; fi
    echo "gpus $g $l: $(grep '^{' $O/g${g}_$l.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["param_hash_per_rank"], d["config"]["loss"])')"
  done
done
