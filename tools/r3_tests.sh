#!/bin/bash
# Round-3 new-path tests: fp16 engines + C4 at B=32 vs oracle, fused streaming hop + C5 pin,
# then the C4 bench line and C5 stream-bench lines.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3t
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "gemm8 or halo or direct_against" > $O/gt_engines.log 2>&1
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_streaming.py -x -v -s --timeout 600 --timeout-method thread > $O/gt_stream.log 2>&1
timeout -k 10 900 python -u -m pytest $R/tests/test_gpu_c4.py -x -v -s --timeout 900 --timeout-method thread > $O/gt_c4.log 2>&1
timeout -k 10 300 python $R/bench.py --spkd --no-cpu-baseline > $O/b_c4_fp16.log 2>&1
timeout -k 10 300 python $R/bench.py --spkd --no-cpu-baseline --precision mixed > $O/b_c4_bf16.log 2>&1
for e in fused graph; do
  for n in 1 64; do
    timeout -k 10 300 python $R/tools/stream_bench.py --engine $e --streams $n > $O/sb_${e}_$n.log 2>&1
  done
done
timeout -k 10 300 python $R/tools/stream_bench.py --engine fused --streams 256 > $O/sb_fused_256.log 2>&1
MODE=fwd timeout -k 10 200 python $R/tools/host_profile.py 10 60 > $O/host_profile.txt 2>&1
echo done
