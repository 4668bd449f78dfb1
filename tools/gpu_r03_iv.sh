# GPU suite (intervals + local references), then the headline bench at 10k and 1,250 documents
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03iv
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc $rc" >> $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="--no-tree-leg --no-node-leg --no-local-leg --no-cpu-baseline"
timeout -k 10 200 python bench.py $B > $O/bench_10k.json 2> $O/bench_10k.err
