set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03verify
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > gpurun_out/r03verify/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-node-leg --no-local-leg --no-tree-leg > gpurun_out/r03verify/bench.json 2> gpurun_out/r03verify/bench.err || exit 1
timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline --no-local-leg --no-tree-leg > gpurun_out/r03verify/bench5.json 2> gpurun_out/r03verify/bench5.err || exit 1
