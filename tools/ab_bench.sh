#!/bin/bash
# A/B of environment knobs on the default bench line: each "NAME=VAL ..." group in $CASES runs
# bench.py once (separate processes; the medians of two passes are printed by the caller).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab
mkdir -p $O
i=0
for pass in ${PASSES:-1 2}; do
  i=0
  IFS=';' read -ra CS <<< "$CASES"
  for c in "${CS[@]}"; do
    i=$((i+1))
    env $c timeout -k 10 120 python $R/bench.py --no-cpu-baseline --steps 20 > $O/c${i}_p$pass.log 2>&1
  done
done
echo ok
