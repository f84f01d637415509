#!/bin/bash
# Round 4 iteration (6): the full GPU suite with the split-product student as the 'mixed' default,
# the driver's default bench line, and student split A/B (back to back, one box).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-r4i}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: rc=$rc"; exit $rc; fi; }
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline"
rc=0; timeout -k 10 600 python -u -m pytest $R/tests -m gpu -v --maxfail=30 --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || rc=$?
tail -3 $O/gpu_suite.log; ok $rc
rc=0; timeout -k 10 170 python $R/bench.py > $O/bench_default.log 2>&1 || rc=$?; ok $rc
for leg in s0:CLSKD_STUDENT_SPLIT=0 s1: s0b:CLSKD_STUDENT_SPLIT=0 s1b:; do
  name=${leg%%:*}; envs=${leg#*:}
  rc=0; env ${envs//,/ } timeout -k 10 150 $B > $O/bench_$name.log 2>&1 || rc=$?; ok $rc
  echo "$name $(grep '^{' $O/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("host_enqueue_ms_per_step"), d.get("serialized_kernel_ms_per_step"), d.get("quality",{}).get("student_wav_rms_vs_fp32_step"))')"
done
grep '^{' $O/bench_default.log | cut -c1-600
echo iter-done
