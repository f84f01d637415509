#!/bin/bash
# C5: fused-hop parity tests, then stream bench lines (fused vs graph).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c5
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_streaming.py -x -v -s --timeout 600 --timeout-method thread > $O/gt.log 2>&1
for n in 1 16 64 256; do
  timeout -k 10 300 python $R/tools/stream_bench.py --engine fused --streams $n > $O/sb_fused_$n.log 2>&1
done
timeout -k 10 300 python $R/tools/stream_bench.py --engine graph --streams 1 > $O/sb_graph_1.log 2>&1
timeout -k 10 300 python $R/tools/hop_marks.py --streams 1 > $O/marks_1.log 2>&1
timeout -k 10 300 python $R/tools/hop_marks.py --streams 256 > $O/marks_256.log 2>&1
cat $O/marks_1.log $O/marks_256.log
tail -q -n 1 $O/sb_*.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/tools/stream_bench.py --engine fused --streams 64 > $O/prof.log 2>&1
find $O/prof -name "*kernel_stats.csv" -exec head -5 {} \;
