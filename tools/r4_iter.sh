#!/bin/bash
# Round 4 iteration on one MI355X: the GPU suite (stops after 10 failures), the driver's default
# bench line, fold on/off A/B (20 steps each), the conv census and a kernel + marker trace of the
# bench (timed region separable: tools/region_stats.py).  Each GPU step has its own time limit;
# a timeout / abort / crash ends the call.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-r4b}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: rc=$rc"; exit $rc; fi; }
rc=0
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -q --maxfail=10 --timeout 600 --timeout-method thread ${TESTS:-} > $O/gpu_tests.log 2>&1 || rc=$?
tail -5 $O/gpu_tests.log
ok $rc
if [ -n "${TESTS_ONLY:-}" ]; then exit 0; fi
rc=0; timeout -k 10 300 python $R/bench.py > $O/bench.log 2>&1 || rc=$?; ok $rc
grep "^{" $O/bench.log | cut -c1-400
rc=0; CLSKD_BN_FOLD=0 timeout -k 10 300 python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_nofold.log 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 300 python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_fold.log 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 200 python $R/tools/conv_census.py > $O/census.txt 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_G8_PP=1 timeout -k 10 200 python $R/tools/conv_census.py > $O/census_pp.txt 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_G8_PP=1 timeout -k 10 300 python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_pp.log 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_F32_SPLIT=1 timeout -k 10 200 python $R/tools/conv_census.py > $O/census_split.txt 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_F32_SPLIT=1 timeout -k 10 300 python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_split.log 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_LSTM_PRIO=1 timeout -k 10 300 python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_lprio.log 2>&1 || rc=$?; ok $rc
rc=0; CLSKD_LSTM_PRIO=1 CLSKD_F32_SPLIT=1 CLSKD_G8_PP=1 timeout -k 10 300 python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_all.log 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 200 python $R/tools/host_profile.py > $O/host_profile.txt 2>&1 || rc=$?; ok $rc
cd /tmp && export TMPDIR=/tmp
rc=0; timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/trace.log 2>&1 || rc=$?; ok $rc
python3 $R/tools/region_stats.py $O/trace/run 20 $O/region_stats.json > $O/region_stats.txt 2>&1 || true
echo iter-done
