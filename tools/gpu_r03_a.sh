set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc $rc" >> $O/gpu_tests.log
# test failures (rc 1) still let the benches run; a crash, fault or time limit stops here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="--steps 10 --warmup 3 --no-tree-leg --no-node-leg --no-local-leg --no-cpu-baseline"
timeout -k 10 200 python bench.py $B > $O/base_10k.json 2> $O/base_10k.err && \
timeout -k 10 200 python bench.py $B --docs 1250 > $O/base_1250.json 2> $O/base_1250.err && \
for v in w4 w5o w4o; do
  MTE_LIB_DIR=build_var/$v timeout -k 10 200 python bench.py $B > $O/${v}_10k.json 2> $O/${v}_10k.err || exit 1
  MTE_LIB_DIR=build_var/$v timeout -k 10 200 python bench.py $B --docs 1250 > $O/${v}_1250.json 2> $O/${v}_1250.err || exit 1
done
