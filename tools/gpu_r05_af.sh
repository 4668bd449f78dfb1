#!/bin/bash
# round 5: apply-kernel waves-per-SIMD floors (build_var/w4, w5) against the product, config 5
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r05af}
mkdir -p $O
P="python3 -u bench.py --config 5 --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg"
timeout -k 10 300 $P > $O/base.json 2> $O/base.err || exit 1
MTE_LIB_DIR=build_var/w4 timeout -k 10 300 $P > $O/w4.json 2> $O/w4.err || exit 1
MTE_LIB_DIR=build_var/w5 timeout -k 10 300 $P > $O/w5.json 2> $O/w5.err || exit 1
