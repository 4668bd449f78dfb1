# round 4, first box: the GPU suite on the current tree, smoke, a config-3 and a config-5 bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-node-leg --no-local-leg --no-tree-leg > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline --no-local-leg --no-tree-leg > $O/bench5.json 2> $O/bench5.err || exit 1
