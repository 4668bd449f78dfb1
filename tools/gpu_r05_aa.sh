#!/bin/bash
# round 5: the reference-farm GPU suites (refs, intervals, reconnect, htree) + a rec trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r05aa}
mkdir -p $O
timeout -k 10 200 node tests/node/interval_farm.js ext > $O/farm_ext.json 2> $O/farm_ext.err || exit 1
timeout -k 10 300 node tests/node/interval_farm.js reconnect > $O/farm_rec.json 2> $O/farm_rec.err || exit 1
MTE_FARM_TRACE=5,1 timeout -k 10 200 node tests/node/interval_farm.js reconnect 6 > $O/t_rec.json 2> $O/t_rec.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_local_refs.py tests/test_intervals.py tests/test_htree.py tests/test_reconnect.py tests/test_local_ops.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" > $O/rc.txt
