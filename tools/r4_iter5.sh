#!/bin/bash
# Round 4 iteration (5): direct channel-lane + split + replay tests, the replay race locator after
# the direct-weight lifetime fix, bench A/B legs, then the full GPU suite with split + channel-lane.
# Every GPU step is bounded below gpurun's 180 s silence limit or writes progress to a file.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-r4g}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: rc=$rc"; exit $rc; fi; }
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline"
rc=0; timeout -k 10 170 python -u -m pytest "$R/tests/test_gpu_parity.py::test_conv_direct_against_torch_and_engine" "$R/tests/test_gpu_parity.py::test_step_graph_matches_eager" "$R/tests/test_gpu_parity.py::test_step_graph_redraws_abf_each_replay" $R/tests/test_gpu_split.py -v --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 || rc=$?
tail -3 $O/gpu_tests.log; ok $rc
rc=0; timeout -k 10 170 python -u $R/tools/race_diag.py --kind exec --replays 6 > $O/race_exec.txt 2>&1 || rc=$?; ok $rc
tail -1 $O/race_exec.txt
for leg in a0: cl:CLSKD_DIRECT_CL=1 split:CLSKD_F32_SPLIT=1 both:CLSKD_F32_SPLIT=1,CLSKD_DIRECT_CL=1 a1:; do
  name=${leg%%:*}; envs=${leg#*:}
  rc=0; env ${envs//,/ } timeout -k 10 150 $B > $O/bench_$name.log 2>&1 || rc=$?; ok $rc
  echo "$name $(grep '^{' $O/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("host_enqueue_ms_per_step"), d.get("serialized_kernel_ms_per_step"))')"
done
rc=0; CLSKD_F32_SPLIT=1 CLSKD_DIRECT_CL=1 timeout -k 10 150 python $R/tools/conv_census.py > $O/census_both.txt 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_F32_SPLIT=1 CLSKD_DIRECT_CL=1 timeout -k 10 600 python -u -m pytest $R/tests -m gpu -v --maxfail=30 --timeout 300 --timeout-method thread > $O/gpu_suite_both.log 2>&1 || rc=$?
tail -3 $O/gpu_suite_both.log; ok $rc
echo iter-done
