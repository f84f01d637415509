#!/bin/bash
# Round 4 iteration (7): re-capture mismatch locator (split student), teacher_ahead A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-r4j}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: rc=$rc"; exit $rc; fi; }
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline"
rc=0; timeout -k 10 170 python -u $R/tools/race_diag.py --kind graph --replays 5 --mutate > $O/race_graph_mut.txt 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_STUDENT_SPLIT=0 timeout -k 10 170 python -u $R/tools/race_diag.py --kind graph --replays 5 --mutate > $O/race_graph_mut_exact.txt 2>&1 || rc=$?; ok $rc
for leg in a0:--no-ahead ahead: a1:--no-ahead ahead2:; do
  name=${leg%%:*}; extra=${leg#*:}
  rc=0; timeout -k 10 150 $B $extra > $O/bench_$name.log 2>&1 || rc=$?; ok $rc
  echo "$name $(grep '^{' $O/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("host_enqueue_ms_per_step"))')"
done
grep "^replay\|differ" $O/race_graph_mut.txt | head -30
echo iter-done
