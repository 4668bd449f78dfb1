# A/B variants of libmte.so (build_var/<name>/, tools/variants.sh) at 10k and 1,250 docs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03var
mkdir -p $O
B="--steps 10 --warmup 3 --no-tree-leg --no-node-leg --no-local-leg --no-cpu-baseline"
for v in "$@"; do
  MTE_LIB_DIR=build_var/$v timeout -k 10 200 python bench.py $B > $O/${v}_10k.json 2> $O/${v}_10k.err || exit 1
  MTE_LIB_DIR=build_var/$v timeout -k 10 200 python bench.py $B --docs 1250 > $O/${v}_1250.json 2> $O/${v}_1250.err || exit 1
done
