#!/bin/bash
# timing-only engine modes need the experiments build: CLSKD_EXPERIMENTS=1 python -m clskd.build (run on the CPU first)
export CLSKD_LIB=exp
# conv_gemm8 iteration: engine parity tests (with CLSKD_G8=$TMODE), then the single-layer
# microbenchmark over the modes in $MODES (CLSKD_G8 = 10*cfg + dbg; 0 = the older engine).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g8
mkdir -p $O
CLSKD_G8=${TMODE:-1} timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "gemm8 or bf16_engine" > $O/gt.log 2>&1
for m in ${MODES:-1 0}; do
  CLSKD_G8=$m timeout -k 10 60 python $R/tools/conv_micro.py --only ${ONLY:-enc2,enc3,enc4,enc5,dec1,dec3,abf3,abf4} > $O/m$m.txt 2>&1
done
echo ok
