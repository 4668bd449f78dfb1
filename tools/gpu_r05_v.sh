#!/bin/bash
# round 5: round-phase parity + config 5 (product, a variant), kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r05v}
V=${VAR:-e2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_chunk.py tests/test_round_sync.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/chunk_tests.log 2>&1 || exit 1
P="python3 bench.py --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg"
timeout -k 10 300 $P --config 5 > $O/bench5.json 2> $O/bench5.err || exit 1
MTE_LIB_DIR=build_var/$V MTE_DIAG_BUILD=1 timeout -k 10 300 $P --config 5 > $O/bench5_$V.json 2> $O/bench5_$V.err || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/stats5 -o run --output-format csv -- $P --config 5 > $O/stats5.json 2> $O/stats5.err || exit 1
echo done > $O/rc.txt
