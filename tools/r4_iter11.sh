#!/bin/bash
# Round 4 iteration (11): C3 captured training step (TrainStepGraph): parity, then the C3 line
# with the capture (default) and eager, then the C2 default line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-r4o}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: rc=$rc"; exit $rc; fi; }
T="python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread"
rc=0; timeout -k 10 300 $T $R/tests/test_gpu_train_graph.py > $O/t_train.log 2>&1 || rc=$?
echo "train tests rc=$rc: $(tail -1 $O/t_train.log)"; ok $rc
grep -m3 "Error:\|assert " $O/t_train.log
rc=0; timeout -k 10 300 $T $R/tests/test_gpu_parity.py -k "step_graph or exec or abf" > $O/t_graph.log 2>&1 || rc=$?
echo "C2 graph tests rc=$rc: $(tail -1 $O/t_graph.log)"; ok $rc
for leg in exec: graph:--launch=graph eager:--launch=eager; do
  name=${leg%%:*}; extra=${leg#*:}
  rc=0; timeout -k 10 170 python $R/bench.py --train --no-cpu-baseline --steps 20 --warmup 3 $extra > $O/train_$name.log 2>&1 || rc=$?; ok $rc
  echo "train $name $(grep '^{' $O/train_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("host_enqueue_ms_per_step"), d["config"]["loss"], d["config"]["launch"][:50])')"
done
echo iter-done
