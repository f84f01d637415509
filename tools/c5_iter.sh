#!/bin/bash
# C5: fused-hop parity tests, then stream bench lines (fused vs graph, 1 and 64 streams).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c5
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_streaming.py -x -v -s --timeout 600 --timeout-method thread > $O/gt.log 2>&1
for e in fused graph; do
  for n in 1 64; do
    timeout -k 10 300 python $R/tools/stream_bench.py --engine $e --streams $n > $O/sb_${e}_$n.log 2>&1
  done
done
timeout -k 10 300 python $R/tools/stream_bench.py --engine fused --streams 256 > $O/sb_fused_256.log 2>&1
tail -n 1 $O/sb_*.log
