#!/bin/bash
# conv_gemm8 K-tile visiting order A/B (CLSKD_G8_KORDER = 1 channel-block-major | 0 packed
# tap-major): engine parity tests, single-layer microbenchmark, FETCH_SIZE of the micro, C2 bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/korder
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "gemm8 or bf16_engine" > $O/gt.log 2>&1
for m in 1 0; do
  CLSKD_G8_KORDER=$m timeout -k 10 90 python $R/tools/conv_micro.py --iters 20 --only enc2,enc3,enc4,enc5,dec1,dec3,abf3,abf4 > $O/m$m.txt 2>&1
  (cd /tmp && export TMPDIR=/tmp && CLSKD_G8_KORDER=$m timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$m -o run -- python3 $R/tools/conv_micro.py --iters 3 --only enc3,enc4,dec1,dec3 > $O/f$m.log 2>&1)
  CLSKD_G8_KORDER=$m timeout -k 10 200 python $R/bench.py --no-cpu-baseline --steps 20 > $O/b$m.log 2>&1
done
echo ok
