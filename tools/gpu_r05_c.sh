#!/bin/bash
# round 5: diagnostic -- pass 1 without the payload planes (wrong digests, timing only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05c
mkdir -p $O
P="python3 bench.py --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg"
for v in np; do
  D=build_var/$v
  MTE_DIAG_BUILD=1 MTE_LIB_DIR=$D timeout -k 10 200 $P --docs 1250 > $O/b1250_$v.json 2> $O/b1250_$v.err || exit 1
  MTE_DIAG_BUILD=1 MTE_LIB_DIR=$D timeout -k 10 200 $P > $O/b3_$v.json 2> $O/b3_$v.err || exit 1
done
echo done > $O/rc.txt
