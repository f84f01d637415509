#!/bin/bash
# Round 4, first GPU call: the GPU suite, the driver's default bench line, a kernel + roctx
# marker trace of bench.py --steps 20 --warmup 5 (timed region separable: tools/region_stats.py),
# SQ/MFMA counters of the dominant conv_gemm8 kernel (one rocprofv3 pass per counter group) and
# the "what if this family were free" sweep (experiments build).  Each GPU step has its own
# time limit; the chain stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4a
mkdir -p $O
rc=0
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -q --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || rc=$?
tail -5 $O/gpu_tests.log
# test failures (rc 1) do not stop the measurements; a timeout / abort / crash does
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python $R/bench.py > $O/bench.log 2>&1
tail -c 600 $O/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/trace.log 2>&1
python3 $R/tools/region_stats.py $O/trace/run 20 $O/region_stats.json > $O/region_stats.txt 2>&1 || true
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  rc=0
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex conv_gemm8 --output-format csv -d $O/sq$i -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/sq$i.log 2>&1 || rc=$?
  echo "pmc pass $i rc=$rc"
  # a killed / timed-out pass ends the GPU work of this call
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit 1; fi
done
cd $R
# A/B: the folded BatchNorm finalize off (fused partials + clskd_bn_finalize launches)
CLSKD_BN_FOLD=0 timeout -k 10 300 python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_nofold.log 2>&1 || echo "nofold bench rc=$?"
timeout -k 10 300 python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_fold.log 2>&1 || echo "fold bench rc=$?"
timeout -k 10 200 python $R/tools/conv_census.py > $O/census.txt 2>&1 || echo "census rc=$?"
bash $R/tools/skip_sweep.sh "0 1 2 32 4 64 8 16 128 0" > $O/skip.log 2>&1 || true
cp -r $R/gpurun_out/skip $O/skip || true
echo r4a-done
