#!/bin/bash
# Round 4 iteration (3): targeted GPU tests, the replay race locator, split-product bench A/B and
# census.  Each GPU step has its own time limit; a timeout / abort / crash ends the call.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-r4e}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: rc=$rc"; exit $rc; fi; }
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline"
rc=0; timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_split.py $R/tests/test_gpu_bnfold.py "$R/tests/test_gpu_parity.py::test_step_graph_matches_eager" "$R/tests/test_gpu_parity.py::test_step_graph_redraws_abf_each_replay" -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || rc=$?
tail -5 $O/gpu_tests.log; ok $rc
rc=0; timeout -k 10 300 python -u $R/tools/race_diag.py --kind exec --replays 8 > $O/race_exec.txt 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 300 python -u $R/tools/race_diag.py --kind graph --replays 8 > $O/race_graph.txt 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 200 $B > $O/bench_a0.log 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_F32_SPLIT=1 timeout -k 10 200 $B > $O/bench_split.log 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 200 $B > $O/bench_a1.log 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_F32_SPLIT=1 timeout -k 10 200 $B > $O/bench_split2.log 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_F32_SPLIT=1 timeout -k 10 200 python $R/tools/conv_census.py > $O/census_split.txt 2>&1 || rc=$?; ok $rc
for f in $O/bench_*.log; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("host_enqueue_ms_per_step"), d.get("serialized_kernel_ms_per_step"))')"; done
echo iter-done
