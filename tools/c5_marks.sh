#!/bin/bash
# C5 fused-hop phase marks only (experiments library): quick A/B of kernel changes.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c5
mkdir -p $O
timeout -k 10 300 python $R/tools/hop_marks.py --streams 1 > $O/marks_1.log 2>&1
timeout -k 10 300 python $R/tools/hop_marks.py --streams 256 > $O/marks_256.log 2>&1
grep -v amdgpu.ids $O/marks_1.log $O/marks_256.log
