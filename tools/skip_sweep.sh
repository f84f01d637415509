#!/bin/bash
# "What if this kernel family were free": C2 eager step time with one family skipped at a time
# (CLSKD_SKIP bit mask, experiments build; results are wrong, only the step time is read).
# Ranks the levers on the real four-stream step.  Diagnostic.
#   bash tools/skip_sweep.sh ["0 1 2 4 ..."]
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/skip
mkdir -p $O
: > $O/summary.txt
for m in ${1:-0 1 2 3 4 8 16 32 64 128 0}; do
  CLSKD_LIB=exp CLSKD_SKIP=$m timeout -k 10 150 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    > $O/b_$m.log 2>&1 || { echo "skip=$m failed rc=$?" >> $O/summary.txt; tail -5 $O/b_$m.log; exit 1; }
  python3 -c "
import json,sys
l=[x for x in open('$O/b_$m.log') if x.startswith('{')][-1]
d=json.loads(l); print('skip=%-4s ms_per_step %.3f' % ('$m', d['ms_per_step']))" >> $O/summary.txt
  tail -1 $O/summary.txt
done
