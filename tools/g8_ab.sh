#!/bin/bash
# conv_gemm8 product-variant A/B (CLSKD_G8 = 1 default | 2 interleaved DMA issue): engine parity
# tests under the variant, then the single-layer microbenchmark for each mode in $MODES.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g8ab
mkdir -p $O
CLSKD_G8=${TMODE:-2} timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "gemm8 or bf16_engine" > $O/gt.log 2>&1
for m in ${MODES:-1 2}; do
  CLSKD_G8=$m timeout -k 10 90 python $R/tools/conv_micro.py --only ${ONLY:-enc2,enc3,enc4,enc5,dec1,dec3,abf3,abf4} > $O/m$m.txt 2>&1
done
for m in ${MODES:-1 2}; do
  CLSKD_G8=$m timeout -k 10 200 python $R/bench.py --no-cpu-baseline --steps 20 > $O/b$m.log 2>&1
done

echo ok
