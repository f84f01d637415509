#!/bin/bash
# Full GPU suite with the channel-block-major K order in both engines, then the C2 conv census,
# FETCH_SIZE of one census pass, and the C2 / C3 bench lines for CLSKD_G8_KORDER = 1 and 0.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/korder2
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gt.log 2>&1
for m in 1 0; do
  CLSKD_G8_KORDER=$m timeout -k 10 120 python $R/tools/conv_census.py > $O/census$m.txt 2>&1
  CLSKD_G8_KORDER=$m timeout -k 10 200 python $R/bench.py --no-cpu-baseline --steps 20 > $O/b$m.log 2>&1
  CLSKD_G8_KORDER=$m timeout -k 10 200 python $R/bench.py --train --no-cpu-baseline --steps 10 > $O/t$m.log 2>&1
  (cd /tmp && export TMPDIR=/tmp && CLSKD_G8_KORDER=$m timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$m -o run -- python3 $R/tools/conv_census.py > $O/f$m.log 2>&1)
done
echo ok
