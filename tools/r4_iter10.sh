#!/bin/bash
# Round 4 iteration (10): conv_halow (staged 16-B epilogue, padded halo rows) parity + per-layer
# A/B vs conv_gemm8; the C3 executor test.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-r4m}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: rc=$rc"; exit $rc; fi; }
T="python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread"
rc=0; timeout -k 10 240 $T $R/tests/test_gpu_parity.py -k "gemm8_against_torch" > $O/t_wide.log 2>&1 || rc=$?
echo "wide tests rc=$rc: $(tail -1 $O/t_wide.log)"; ok $rc
[ $rc -eq 0 ] || { grep -m5 "Error\|assert" $O/t_wide.log; exit 1; }
L=enc2,enc3,enc4,enc5,dec1,dec3,abf3,abf4
for hw in 1 0; do
  rc=0; CLSKD_HALOW=$hw timeout -k 10 150 python -u $R/tools/conv_micro.py --iters 30 --only $L > $O/micro_hw$hw.txt 2>&1 || rc=$?; ok $rc
done
paste <(grep TF $O/micro_hw1.txt) <(grep TF $O/micro_hw0.txt | awk '{print $(NF-3), $(NF-1)}')
rc=0; timeout -k 10 300 $T -s $R/tests/test_gpu_train_graph.py > $O/t_train.log 2>&1 || rc=$?
echo "train tests rc=$rc: $(tail -1 $O/t_train.log)"; ok $rc
grep -m3 "Error\|assert\|executor:" $O/t_train.log
echo iter-done
