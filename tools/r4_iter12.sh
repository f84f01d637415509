#!/bin/bash
# Round 4 iteration (12): concurrent-step grid cap — parity (bitwise vs the full grid, step
# graph / executor, teacher_ahead, the C2 oracle test), then the C2 line with and without.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-r4q}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: rc=$rc"; exit $rc; fi; }
T="python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread"
rc=0; timeout -k 10 400 $T $R/tests/test_gpu_parity.py -k "grid_cap or step_graph or teacher_ahead or clskd_step" $R/tests/test_gpu_c2_mixed.py > $O/t.log 2>&1 || rc=$?
echo "tests rc=$rc: $(tail -1 $O/t.log)"; ok $rc
[ $rc -eq 0 ] || { grep -m5 "Error\|assert" $O/t.log; exit 1; }
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for leg in cap1:0.875 full1:0 cap2:0.875 full2:0 cap3:0.875 full3:0; do
  name=${leg%%:*}; fr=${leg#*:}
  rc=0; CLSKD_STEP_G8_GRID_FRAC=$fr timeout -k 10 150 $B > $O/b_$name.log 2>&1 || rc=$?; ok $rc
  echo "$name $(grep '^{' $O/b_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["host_enqueue_ms_per_step"])')"
done
echo iter-done
