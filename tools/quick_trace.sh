set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/gq
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread -k "gram or spkd or step or loss" > $O/t.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/trace.log 2>&1
echo ok
