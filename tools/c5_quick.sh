#!/bin/bash
# C5 fused hop: parity tests + phase marks (1 and 256 streams) + one stream_bench line.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c5
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_streaming.py -x -v -s --timeout 600 --timeout-method thread > $O/gt.log 2>&1
grep -E "max \|diff" $O/gt.log | cut -c1-150
timeout -k 10 300 python $R/tools/hop_marks.py --streams 1 > $O/marks_1.log 2>&1
timeout -k 10 300 python $R/tools/hop_marks.py --streams 256 > $O/marks_256.log 2>&1
grep -h -E "fused hop|shader" $O/marks_1.log $O/marks_256.log
timeout -k 10 300 python $R/tools/stream_bench.py --engine fused --streams 256 > $O/sb_fused_256.log 2>&1
timeout -k 10 300 python $R/tools/stream_bench.py --engine fused --streams 1 > $O/sb_fused_1.log 2>&1
grep -h -o '"streams": [0-9]*\|"ms_per_hop": [0-9.]*\|"frames_per_second": [0-9.]*' $O/sb_fused_1.log $O/sb_fused_256.log | paste - - -
