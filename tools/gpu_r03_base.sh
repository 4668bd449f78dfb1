set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03base
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03base/gpu_tests.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg > gpurun_out/r03base/bench.json 2> gpurun_out/r03base/bench.err && \
timeout -k 10 200 python bench.py --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg --docs 1250 > gpurun_out/r03base/bench1250.json 2> gpurun_out/r03base/bench1250.err
