#!/bin/bash
# round 4: where the HBM tree pass's time goes on the local-client line:
# doc-count sweep (chain- or throughput-bound), phase clocks, issue counters
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 300 python -u tools/lc_probe.py > $O/probe.json 2> $O/probe.err || exit 1
timeout -k 10 300 python -u tools/local_leg.py --prof 0 > $O/prof.json 2> $O/prof.err || exit 1
cp gpurun_out/htree_prof_0.txt $O/ 2>/dev/null
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --kernel-trace -d $O/pmc_issue -o run --output-format csv -- python3 tools/local_leg.py 0 > $O/pmc_issue.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INSTS_FLAT --kernel-trace -d $O/pmc_mem -o run --output-format csv -- python3 tools/local_leg.py 0 > $O/pmc_mem.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 tools/local_leg.py 0 > $O/stats.log 2>&1 || exit 1
echo done > $O/rc.txt
