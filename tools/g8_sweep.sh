#!/bin/bash
# timing-only engine modes need the experiments build: CLSKD_EXPERIMENTS=1 python -m clskd.build (run on the CPU first)
export CLSKD_LIB=exp
# conv_gemm8 configuration / ablation sweep (CLSKD_G8=<cfg*10+dbg>) on the wide teacher layers.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g8s
mkdir -p $O
for m in ${MODES:-1 10 11 12 13 20 30 40 0}; do
  CLSKD_G8=$m timeout -k 10 60 python $R/tools/conv_micro.py --only ${ONLY:-enc3,enc4,dec1,dec3,abf3,abf4} > $O/m$m.txt 2>&1
done
echo ok
