#!/bin/bash
# Halo-tiled fp32 kernel on the 8/16-wide student decoder layers (CLSKD_HALO32_MIN_N=8) vs the
# fp32 engine (default 32): parity tests, the C2 conv census, C2 and C3 bench lines per setting.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/h32n
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "halo_f32" > $O/gt.log 2>&1
for m in 32 8; do
  CLSKD_HALO32_MIN_N=$m timeout -k 10 120 python $R/tools/conv_census.py > $O/census$m.txt 2>&1
  CLSKD_HALO32_MIN_N=$m timeout -k 10 200 python $R/bench.py --no-cpu-baseline --steps 20 > $O/b$m.log 2>&1
  CLSKD_HALO32_MIN_N=$m timeout -k 10 200 python $R/bench.py --train --no-cpu-baseline --steps 10 > $O/t$m.log 2>&1
done
echo ok
