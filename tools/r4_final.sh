#!/bin/bash
# Round-4 end evidence on one MI355X (via gpurun from the repo root): the GPU suite; two PMC passes of the bench
# (FETCH_SIZE, WRITE_SIZE separately) joined by tools/pmc_traffic.py; a rocprofv3 kernel + marker
# trace of the driver's bench command split at its roctx ranges (tools/region_stats.py: census
# step and timed steps separately); the default bench line; the C3 / C4 / C1 / C5 lines.  Every
# GPU step has its own time limit; a timeout / abort / crash ends the call.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-r4final}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "stop: rc=$rc"; exit $rc; fi; }
rc=0; timeout -k 10 400 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 || rc=$?; ok $rc
tail -2 $O/gpu_suite.log
(
  cd /tmp && export TMPDIR=/tmp
  rc=0; timeout -k 10 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch.log 2>&1 || rc=$?; ok $rc
  rc=0; timeout -k 10 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/write.log 2>&1 || rc=$?; ok $rc
  rc=0; timeout -k 10 170 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/trace.log 2>&1 || rc=$?; ok $rc
) || exit $?
python3 $R/tools/pmc_traffic.py $O/fetch/run_counter_collection.csv $O/write/run_counter_collection.csv $O/r4_pmc_traffic.json > $O/traffic.txt
python3 $R/tools/region_stats.py $O/trace/run 20 $O/r4_region_stats.json > $O/region_stats.txt 2>&1 || true
rc=0; timeout -k 10 170 python $R/bench.py > $O/bench.log 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 170 python $R/bench.py --train --no-cpu-baseline > $O/bench_train.log 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 170 python $R/bench.py --spkd --no-cpu-baseline > $O/bench_spkd.log 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 170 python $R/bench.py --c1 > $O/bench_c1.log 2>&1 || rc=$?; ok $rc
rc=0; timeout -k 10 170 python $R/bench.py --c5 > $O/bench_c5.log 2>&1 || rc=$?; ok $rc
for f in $O/bench*.log; do echo "$f $(grep '^{' $f | cut -c1-200)"; done
echo final-done
