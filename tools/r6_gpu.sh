#!/bin/bash
# Round-6 GPU call (from the repo root via gpurun).  STEPS selects what runs (space separated):
#   suite   full GPU suite (+ the C3 gradient-parity table written to $O/c3_grad_parity.txt)
#   bench   default C2 bench line;  train  C3 line;  spkd  C4 line;  c1 / c5
#   trace   rocprofv3 kernel+marker trace of the bench command split at its roctx ranges
#   pmc     FETCH_SIZE / WRITE_SIZE passes -> per-kernel HBM traffic
#   tests:<pytest args>   a subset of the suite (comma-separated)
# Every GPU step has its own time limit; a failing step ends the call.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-r6}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "stop: rc=$rc ($2)"; exit $rc; fi; }
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
for st in ${STEPS:-suite bench}; do
  case $st in
    suite)
      rc=0; CLSKD_GRAD_PARITY_OUT=$O/c3_grad_parity.txt timeout -k 10 900 $T $R/tests -m gpu > $O/gpu_suite.log 2>&1 || rc=$?
      tail -2 $O/gpu_suite.log; ok $rc suite;;
    tests:*)
      a=${st#tests:}; rc=0; timeout -k 10 600 $T -m gpu ${a//,/ } > $O/tests.log 2>&1 || rc=$?
      tail -2 $O/tests.log; ok $rc tests;;
    bench) rc=0; timeout -k 10 300 python $R/bench.py $BENCH_ARGS > $O/bench.log 2>&1 || rc=$?; ok $rc bench
      grep '^{' $O/bench.log | cut -c1-400;;
    train) rc=0; timeout -k 10 300 python $R/bench.py --train --no-cpu-baseline > $O/bench_train.log 2>&1 || rc=$?; ok $rc train
      grep '^{' $O/bench_train.log | cut -c1-300;;
    spkd) rc=0; timeout -k 10 300 python $R/bench.py --spkd --no-cpu-baseline > $O/bench_spkd.log 2>&1 || rc=$?; ok $rc spkd;;
    c1) rc=0; timeout -k 10 300 python $R/bench.py --c1 > $O/bench_c1.log 2>&1 || rc=$?; ok $rc c1;;
    c5) rc=0; timeout -k 10 300 python $R/bench.py --c5 > $O/bench_c5.log 2>&1 || rc=$?; ok $rc c5;;
    trace)
      ( cd /tmp && export TMPDIR=/tmp
        rc=0; timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $BENCH_ARGS > $O/trace.log 2>&1 || rc=$?; ok $rc trace ) || exit $?
      python3 $R/tools/region_stats.py $O/trace/run 20 $O/region_stats.json > $O/region_stats.txt 2>&1 || true
      grep '^{' $O/trace.log | cut -c1-300;;
    pmc)
      ( cd /tmp && export TMPDIR=/tmp
        rc=0; timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch.log 2>&1 || rc=$?; ok $rc fetch
        rc=0; timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/write.log 2>&1 || rc=$?; ok $rc write ) || exit $?
      python3 $R/tools/pmc_traffic.py $O/fetch/run_counter_collection.csv $O/write/run_counter_collection.csv $O/pmc_traffic.json > $O/traffic.txt;;
    pmc_train)  # the C3 leg's own FETCH_SIZE / WRITE_SIZE passes (round 6: the C3 line's traffic)
      ( cd /tmp && export TMPDIR=/tmp
        rc=0; timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/tfetch -o run -- python3 $R/bench.py --train --steps 2 --warmup 2 --no-cpu-baseline > $O/tfetch.log 2>&1 || rc=$?; ok $rc tfetch
        rc=0; timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/twrite -o run -- python3 $R/bench.py --train --steps 2 --warmup 2 --no-cpu-baseline > $O/twrite.log 2>&1 || rc=$?; ok $rc twrite ) || exit $?
      python3 $R/tools/pmc_traffic.py $O/tfetch/run_counter_collection.csv $O/twrite/run_counter_collection.csv $O/train_pmc_traffic.json > $O/train_traffic.txt;;
    sq)  # MFMA utilisation / wait counters of the conv_gemm8 instances inside the C2 bench: three
         # --pmc passes (the per-block slot limits), kernel filter, summarised by tools/sq_summary.py
      ( cd /tmp && export TMPDIR=/tmp; i=0
        for P in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES" \
                 "SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_MOPS_BF16" \
                 "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
          i=$((i+1)); rc=0
          timeout -s KILL 200 rocprofv3 --pmc $P --kernel-include-regex conv_gemm8 --output-format csv -d $O/sq$i -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sq$i.log 2>&1 || rc=$?
          ok $rc sq$i
        done ) || exit $?
      python3 $R/tools/sq_summary.py $O/g8_counters.json $O/sq1/run_counter_collection.csv $O/sq2/run_counter_collection.csv $O/sq3/run_counter_collection.csv > $O/sq_summary.txt 2>&1 || true
      tail -5 $O/sq_summary.txt;;
    micro) rc=0; timeout -k 10 300 python $R/tools/conv_micro.py $MICRO_ARGS > $O/micro.log 2>&1 || rc=$?; cat $O/micro.log; ok $rc micro;;
    ab)  # same-box A/B on the C2 line: AB_CASES="A=1 B=2;A=0 :: --launch exec" (';'-separated
         # cases: env assignments, optionally '::' and extra bench.py arguments)
      IFS=';' read -ra CS <<< "$AB_CASES"
      for pass in 1 2 3; do
        i=0
        for c in "${CS[@]}"; do
          i=$((i+1)); rc=0
          ce=${c%%::*}; ca=""; [[ "$c" == *::* ]] && ca=${c#*::}
          env $ce timeout -k 10 200 python $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 $BENCH_ARGS $ca > $O/ab_c${i}_p$pass.log 2>&1 || rc=$?; ok $rc ab
          echo "[$c] pass $pass: $(grep '^{' $O/ab_c${i}_p$pass.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], "ms, host", d["host_enqueue_ms_per_step"], "frac", r["frac"], r.get("kernel"), r.get("isolated_avg_launch_us"), "census", r.get("all_kernels_isolated", {}).get("ms_per_step"))')"
        done
      done;;
    ab2)  # a second same-box A/B in the same call: AB2_CASES / BENCH2_ARGS (as ab)
      IFS=';' read -ra CS <<< "$AB2_CASES"
      for pass in 1 2 3; do
        i=0
        for c in "${CS[@]}"; do
          i=$((i+1)); rc=0
          ce=${c%%::*}; ca=""; [[ "$c" == *::* ]] && ca=${c#*::}
          env $ce timeout -k 10 200 python $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 $BENCH2_ARGS $ca > $O/ab2_c${i}_p$pass.log 2>&1 || rc=$?; ok $rc ab2
          echo "[$c] pass $pass: $(grep '^{' $O/ab2_c${i}_p$pass.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], "ms, host", d["host_enqueue_ms_per_step"], "frac", r["frac"], r.get("kernel"), r.get("isolated_avg_launch_us"), "census", r.get("all_kernels_isolated", {}).get("ms_per_step"))')"
        done
      done;;
    hostprof) rc=0; timeout -k 10 300 python $R/tools/host_profile.py --steps 20 --top 60 > $O/hostprof.txt 2>&1 || rc=$?; ok $rc hostprof
      head -3 $O/hostprof.txt;;
    trace_train_exec)
      ( cd /tmp && export TMPDIR=/tmp
        rc=0; timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $O/tetrace -o run -- python3 $R/bench.py --train --launch exec --steps 10 --warmup 3 --no-cpu-baseline > $O/tetrace.log 2>&1 || rc=$?; ok $rc trace_train_exec ) || exit $?
      python3 $R/tools/region_stats.py $O/tetrace/run 10 $O/train_exec_region_stats.json > $O/train_exec_region_stats.txt 2>&1 || true
      grep '^{' $O/tetrace.log | cut -c1-300;;
    trace_train)
      ( cd /tmp && export TMPDIR=/tmp
        rc=0; timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $O/ttrace -o run -- python3 $R/bench.py --train --steps 10 --warmup 3 --no-cpu-baseline > $O/ttrace.log 2>&1 || rc=$?; ok $rc trace_train ) || exit $?
      python3 $R/tools/region_stats.py $O/ttrace/run 10 $O/train_region_stats.json > $O/train_region_stats.txt 2>&1 || true
      grep '^{' $O/ttrace.log | cut -c1-300;;
    py:*) f=${st#py:}; f=${f//,/ }; rc=0; timeout -k 10 300 python $R/$f > $O/py_$(basename ${f%% *} .py).txt 2>&1 || rc=$?
      tail -30 $O/py_$(basename ${f%% *} .py).txt; ok $rc py;;
    abl)  # conv_gemm8 TA ablations (experiments library, CLSKD_G8 = 100 + flags: 1 no DMA, 2 no
          # MFMA, 4 no fragment reads, 8 no epilogue, 16 A pieces only, 32 B only, 64 no DMA wait),
          # all modes interleaved per layer in one process (tools/conv_micro.py --ab)
      rc=0; CLSKD_LIB=exp timeout -k 10 400 python -u $R/tools/conv_micro.py --iters 20 --rounds 3 \
        --only ${ABL_LAYERS:-enc3,enc4,enc5,dec1,dec3,abf3,abf4,pw64k} \
        --ab CLSKD_G8=${ABL_MODES:-100,101,102,103,104,106,107,108,111,115,116,132,164} > $O/abl.txt 2>&1 || rc=$?
      cat $O/abl.txt | grep -v amdgpu.ids; ok $rc abl;;
    skip)  # "what if this kernel family were free" (CLSKD_SKIP bit mask, experiments library,
           # wrong results, step time only): SKIP_MODES interleaved over 3 passes, BENCH_ARGS
           # selects the leg (e.g. --train).  Bits: 8 LSTM recurrence (plain), 256 taped H=32
           # recurrence (lstm_recurrent_pre), 512 LSTM backward, 32 Gram partials
      for pass in 1 2 3; do
        for m in ${SKIP_MODES:-0 8 256 512 776}; do
          rc=0; CLSKD_LIB=exp CLSKD_SKIP=$m timeout -k 10 200 python $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 $BENCH_ARGS > $O/skip_${m}_p$pass.log 2>&1 || rc=$?; ok $rc skip
          echo "skip=$m pass $pass: $(grep '^{' $O/skip_${m}_p$pass.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms")')" | tee -a $O/skip_summary.txt
        done
      done;;
    *) echo "unknown step $st"; exit 2;;
  esac
done
echo r6-done
