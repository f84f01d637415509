#!/bin/bash
# Round-3 GPU test suite (one process, per-test timeout) -> gpurun_out/round/gpu_tests.log
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/round
mkdir -p $O
timeout -k 10 1000 python -u -m pytest $R/tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
exit $rc
