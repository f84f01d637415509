#!/bin/bash
# C3 training step: kernel trace + the two HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE), each
# its own run (tools/pmc_traffic.py joins them).  Diagnostic for the backward's kernels.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/tp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --train --steps 3 --warmup 2 --no-cpu-baseline > $O/trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --train --steps 1 --warmup 1 --no-cpu-baseline > $O/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py --train --steps 1 --warmup 1 --no-cpu-baseline > $O/write.log 2>&1
echo done
