#!/bin/bash
# Round-end evidence on one MI355X (run via gpurun from the repo root; the GPU test suite runs
# separately, tools/r3_tests.sh): two PMC passes of the bench (FETCH_SIZE, WRITE_SIZE
# separately) joined by tools/pmc_traffic.py into profiles/r3_pmc_traffic.json (so the bench
# lines below carry roofline.traffic for the kernel instances of THIS build); the default bench
# line; the C3 training-step, C4 SPKD and C1 lines; a rocprofv3 kernel-trace/stats pass of the
# bench.  Every GPU step has its own time limit; the chain stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/round
mkdir -p $O
(
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/write.log 2>&1
)
python3 $R/tools/pmc_traffic.py $O/fetch/run_counter_collection.csv $O/write/run_counter_collection.csv $R/profiles/r3_pmc_traffic.json > $O/traffic.txt
cp $R/profiles/r3_pmc_traffic.json $O/r3_pmc_traffic.json
timeout -k 10 300 python $R/bench.py > $O/bench.log 2>&1
timeout -k 10 200 python $R/bench.py --train --no-cpu-baseline > $O/bench_train.log 2>&1
timeout -k 10 200 python $R/bench.py --spkd --no-cpu-baseline > $O/bench_spkd.log 2>&1
timeout -k 10 200 python $R/bench.py --c1 > $O/bench_c1.log 2>&1
timeout -k 10 300 python $R/bench.py --c5 > $O/bench_c5.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/trace.log 2>&1
echo done
