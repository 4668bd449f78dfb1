#!/bin/bash
# round 5: chunk fill A/B (build_var/f160, f176) against the product, config 5
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r05am}
mkdir -p $O
P="python3 -u bench.py --config 5 --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg"
timeout -k 10 300 $P > $O/base.json 2> $O/base.err || exit 1
MTE_LIB_DIR=build_var/f160 timeout -k 10 300 $P > $O/f160.json 2> $O/f160.err || exit 1
MTE_LIB_DIR=build_var/f176 timeout -k 10 300 $P > $O/f176.json 2> $O/f176.err || exit 1
