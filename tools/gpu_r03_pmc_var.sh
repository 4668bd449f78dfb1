# HBM traffic (two PMC passes) of pass-1 variants: build_var/<name> libraries
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03pmc
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg --steps 1 --warmup 0"
for v in "$@"; do
  MTE_LIB_DIR=build_var/$v timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/$v/fetch -o run --output-format csv -- $B > $O/$v.fetch.json 2> $O/$v.fetch.err || exit 1
  MTE_LIB_DIR=build_var/$v timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/$v/write -o run --output-format csv -- $B > $O/$v.write.json 2> $O/$v.write.err || exit 1
done
