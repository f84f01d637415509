#!/bin/bash
# Same-box A/B of an environment knob: conv micro + 2 bench runs per arm.
#   bash tools/ab_env.sh VAR "micro-configs"
V=$1; CFG=$2
set -e
for i in 1 2; do
  for val in 0 1; do
    env $V=$val timeout -k 10 150 python tools/conv_micro.py --only $CFG 2>&1 | grep -v amdgpu | sed "s/^/$V=$val /"
    v=$(env $V=$val timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*')
    echo "$V=$val bench $v"
  done
done
