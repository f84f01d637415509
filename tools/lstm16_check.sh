#!/bin/bash
# Teacher LSTM outputs stored 16-bit: full GPU suite (the benched C2 / C4 configurations against
# the oracle are in it), the C2 conv census and C2 / C4 bench lines.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/lstm16
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gt.log 2>&1
timeout -k 10 120 python $R/tools/conv_census.py > $O/census.txt 2>&1
timeout -k 10 200 python $R/bench.py --no-cpu-baseline --steps 20 > $O/b.log 2>&1
timeout -k 10 200 python $R/bench.py --no-cpu-baseline --steps 20 > $O/b2.log 2>&1
timeout -k 10 200 python $R/bench.py --spkd --no-cpu-baseline > $O/s.log 2>&1
echo ok
