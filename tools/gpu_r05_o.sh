#!/bin/bash
# round 5: farms + ref/interval/chunk GPU tests, config 5 (product, diagnostics, kernel stats)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r05o}
mkdir -p $O
timeout -k 10 200 node tests/node/interval_farm.js ext > $O/farm_ext.json 2> $O/farm_ext.err || exit 1
timeout -k 10 300 node tests/node/interval_farm.js reconnect > $O/farm_rec.json 2> $O/farm_rec.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_local_refs.py tests/test_intervals.py tests/test_gpu_chunk.py tests/test_round_sync.py tests/test_nan_merge.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" > $O/rc.txt
P="python3 bench.py --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg"
timeout -k 10 300 $P --config 5 > $O/bench5.json 2> $O/bench5.err || exit 1
MTE_LIB_DIR=build_var/diag MTE_DIAG_BUILD=1 timeout -k 10 300 $P --config 5 --steps 2 --warmup 1 > $O/diag5.json 2> $O/diag5.err || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/stats5 -o run --output-format csv -- $P --config 5 > $O/stats5.json 2> $O/stats5.err || exit 1
echo done >> $O/rc.txt
