# pass-1 step variants: parity first (the GPU parity and round-sync tests on the
# variant library), then the bench at 10k and 1,250 docs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03lean
mkdir -p $O
MTE_LIB_DIR=build_var/lean timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_round_sync.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/lean_parity.log 2>&1
rc=$?; echo "rc $rc" >> $O/lean_parity.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="--steps 10 --warmup 3 --no-tree-leg --no-node-leg --no-local-leg --no-cpu-baseline"
for v in lean w5s; do
  MTE_LIB_DIR=build_var/$v timeout -k 10 200 python bench.py $B > $O/${v}_10k.json 2> $O/${v}_10k.err || exit 1
  MTE_LIB_DIR=build_var/$v timeout -k 10 200 python bench.py $B --docs 1250 > $O/${v}_1250.json 2> $O/${v}_1250.err || exit 1
done
