#!/bin/bash
# round 5: pass-1 stall breakdown at 1,250 documents (one document per wave) and
# at 10k (config 3): two --pmc passes each, <= 8 SQ counters per pass
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r05stall}
mkdir -p $O
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg"
A="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES"
C="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAVE_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $A --kernel-trace -d $O/d1250_a -o run --output-format csv -- $B --docs 1250 > $O/d1250_a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/d1250_c -o run --output-format csv -- $B --docs 1250 > $O/d1250_c.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $A --kernel-trace -d $O/d10k_a -o run --output-format csv -- $B > $O/d10k_a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/d10k_c -o run --output-format csv -- $B > $O/d10k_c.log 2>&1 || exit 1
echo done > $O/rc.txt
