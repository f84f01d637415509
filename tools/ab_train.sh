#!/bin/bash
# A/B of environment knobs on the C3 training-step bench line (bench.py --train), like
# tools/ab_bench.sh.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abt
mkdir -p $O
for pass in ${PASSES:-1 2}; do
  i=0
  IFS=';' read -ra CS <<< "$CASES"
  for c in "${CS[@]}"; do
    i=$((i+1))
    env $c timeout -k 10 150 python $R/bench.py --train --no-cpu-baseline --steps 8 --warmup 3 > $O/c${i}_p$pass.log 2>&1
  done
done
echo ok
