#!/bin/bash
# Round 4 iteration (9): conv_halow (wide-layer halo kernel) parity + per-layer A/B vs conv_gemm8,
# the C3 captured training step, then the C2 / C3 lines.  A test failure (rc 1) is recorded and
# the call goes on; a crash, abort or timeout ends it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-r4l}
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
rc=0; timeout -k 10 400 $T $R/tests/test_gpu_bnfold.py $R/tests/test_gpu_c2_mixed.py $R/tests/test_gpu_train_graph.py > $O/t_more.log 2>&1 || rc=$?
echo "more tests rc=$rc: $(tail -1 $O/t_more.log)"; ok $rc
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for leg in hw1:1 hw0:0 hw1b:1; do
  name=${leg%%:*}; hw=${leg#*:}
  rc=0; CLSKD_HALOW=$hw timeout -k 10 150 $B > $O/bench_$name.log 2>&1 || rc=$?; ok $rc
  echo "$name $(grep '^{' $O/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("host_enqueue_ms_per_step"), d.get("serialized_kernel_ms_per_step"), d["roofline"]["kernel"], d["quality"]["si_snr_delta_db"])')"
done
for leg in exec:--launch=exec eager:--launch=eager; do
  name=${leg%%:*}; extra=${leg#*:}
  rc=0; timeout -k 10 170 python $R/bench.py --train --no-cpu-baseline --steps 20 --warmup 3 $extra > $O/train_$name.log 2>&1 || rc=$?; ok $rc
  echo "train $name $(grep '^{' $O/train_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("host_enqueue_ms_per_step"), d["config"]["loss"])')"
done
echo iter-done
