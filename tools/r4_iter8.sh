#!/bin/bash
# Round 4 iteration (8): C3 captured training step (TrainStepExecutor) — parity tests, then the
# C3 line with the executor (default) and eager, back to back.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-r4k}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "stop: rc=$rc"; exit $rc; fi; }
rc=0; timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_train_graph.py $R/tests/test_gpu_backward.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $O/gt.log 2>&1 || rc=$?
tail -5 $O/gt.log; ok $rc
for leg in exec:--launch=exec eager:--launch=eager exec2:; do
  name=${leg%%:*}; extra=${leg#*:}
  rc=0; timeout -k 10 170 python $R/bench.py --train --no-cpu-baseline --steps 20 --warmup 3 $extra > $O/bench_$name.log 2>&1 || rc=$?; ok $rc
  echo "$name $(grep '^{' $O/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("host_enqueue_ms_per_step"), d["config"]["launch"][:60], d["config"]["loss"])')"
done
echo iter-done
