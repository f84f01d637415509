#!/bin/bash
# Kernel traces of each chain of the C2 step run alone (tools/chain_profile.py).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/chains
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in ${CHAINS:-student rdec renc teacher}; do
  timeout -k 10 120 python3 $R/tools/chain_profile.py $w 5 > $O/$w.txt 2>&1
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$w -o run -- python3 $R/tools/chain_profile.py $w 5 > $O/${w}_prof.log 2>&1
done
echo ok
