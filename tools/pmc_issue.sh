#!/bin/bash
# Issue counters of the replay kernels for one bench configuration (one --pmc
# pass, <= 8 SQ counters): tools/pmc_issue.sh <out_dir> [bench.py args]
set -e
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p $out
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --kernel-trace -d $out -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-tree-leg --no-node-leg "$@" > $out/bench.log 2>&1
