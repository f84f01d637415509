set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/g1
mkdir -p $O
timeout -k 10 500 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gt.log 2>&1
timeout -k 10 300 python $R/bench.py > $O/b.log 2>&1
echo ok
