#!/bin/bash
# Round 4 iteration (4): split-engine tests, the replay race locator (program dump; tag / stream
# variants), split K-tile depth A/B (bench + census).  Each GPU step has its own time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-r4f}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: rc=$rc"; exit $rc; fi; }
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline"
rc=0; timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_split.py "$R/tests/test_gpu_parity.py::test_conv_direct_against_torch_and_engine" -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || rc=$?
tail -3 $O/gpu_tests.log; ok $rc
rc=0; timeout -k 10 200 python -u $R/tools/race_diag.py --kind exec --replays 4 --dump > $O/race_exec_dump.txt 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_EXEC_TAGS=0 timeout -k 10 200 python -u $R/tools/race_diag.py --kind exec --replays 4 > $O/race_exec_notags.txt 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_EXEC_OWN_STREAMS=1 timeout -k 10 200 python -u $R/tools/race_diag.py --kind exec --replays 4 > $O/race_exec_own.txt 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 200 python -u $R/tools/race_diag.py --kind exec --streams 2 --replays 4 > $O/race_exec_s2.txt 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_F32_SPLIT=1 timeout -k 10 200 $B > $O/bench_split64.log 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_F32_SPLIT=1 CLSKD_SPLIT_BK=32 timeout -k 10 200 $B > $O/bench_split32.log 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 200 $B > $O/bench_a0.log 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_DIRECT_CL=1 timeout -k 10 200 $B > $O/bench_cl.log 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_F32_SPLIT=1 CLSKD_DIRECT_CL=1 timeout -k 10 200 $B > $O/bench_split_cl.log 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_F32_SPLIT=1 CLSKD_DIRECT_CL=1 timeout -k 10 200 python $R/tools/conv_census.py > $O/census_split_cl.txt 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_F32_SPLIT=1 CLSKD_DIRECT_CL=1 timeout -k 10 500 python -u -m pytest $R/tests -m gpu -q --maxfail=30 --timeout 300 --timeout-method thread > $O/gpu_suite_split_cl.log 2>&1 || rc=$?
tail -3 $O/gpu_suite_split_cl.log; ok $rc
for f in $O/bench_*.log; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("host_enqueue_ms_per_step"), d.get("serialized_kernel_ms_per_step"))')"; done
for f in $O/race_exec*.txt; do echo "$f: $(tail -1 $f)"; done
echo iter-done
