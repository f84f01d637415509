#!/bin/bash
# Round-3 end: the GPU suite, then the round evidence (tools/round_profile.sh).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/round
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/round/gpu_tests.log 2>&1
bash $R/tools/round_profile.sh
