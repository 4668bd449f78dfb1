#!/bin/bash
# round 5, first call: baseline of the current library at 1,250 documents (the
# N = 8 per-GPU share) and config 3, plus the stall breakdown of pass 1 at
# 1,250 documents (two --pmc passes of 8 SQ counters each)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05a
mkdir -p $O
P="python3 bench.py --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg"
timeout -k 10 300 $P --docs 1250 > $O/bench_1250.json 2> $O/bench_1250.err || exit 1
timeout -k 10 300 $P > $O/bench3.json 2> $O/bench3.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS --kernel-trace -d $O/pmc_a -o run --output-format csv -- $P --docs 1250 --steps 1 --warmup 0 > $O/pmc_a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_WAVES SQ_ACTIVE_INST_MISC --kernel-trace -d $O/pmc_b -o run --output-format csv -- $P --docs 1250 --steps 1 --warmup 0 > $O/pmc_b.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/stats_1250 -o run --output-format csv -- $P --docs 1250 > $O/stats_1250.log 2>&1 || exit 1
echo done > $O/rc.txt
