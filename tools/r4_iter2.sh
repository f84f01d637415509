#!/bin/bash
# Round 4 iteration (2): GPU suite, executor diagnostic, bench A/B legs (default / LSTM priority /
# split-product fp32 / both, then default again: same box, back to back), census with the split
# engine, host profile, and a kernel + marker trace of the default bench.  Each GPU step has its
# own time limit; a timeout / abort / crash ends the call.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-r4d}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: rc=$rc"; exit $rc; fi; }
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline"
rc=0; timeout -k 10 600 python -u -m pytest $R/tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread ${TESTS:-} > $O/gpu_tests.log 2>&1 || rc=$?
tail -5 $O/gpu_tests.log; ok $rc
if [ -n "${TESTS_ONLY:-}" ]; then exit 0; fi
rc=0; timeout -k 10 300 python -u $R/tools/exec_diag.py > $O/exec_diag.txt 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 200 $B > $O/bench_a0.log 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_LSTM_PRIO=1 timeout -k 10 200 $B > $O/bench_lprio.log 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_F32_SPLIT=1 timeout -k 10 200 $B > $O/bench_split.log 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_LSTM_PRIO=1 CLSKD_F32_SPLIT=1 timeout -k 10 200 $B > $O/bench_both.log 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 200 $B > $O/bench_a1.log 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 200 $B --launch exec > $O/bench_exec.log 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_LSTM_PRIO=1 CLSKD_F32_SPLIT=1 timeout -k 10 200 $B --launch exec > $O/bench_exec_both.log 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_F32_SPLIT=1 timeout -k 10 200 python $R/tools/conv_census.py > $O/census_split.txt 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 200 python $R/tools/host_profile.py > $O/host_profile.txt 2>&1 || rc=$?; ok $rc
for f in $O/bench_*.log; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("host_enqueue_ms_per_step"), d.get("serialized_kernel_ms_per_step"))')"; done
echo iter-done
