#!/bin/bash
# round 5: the local-client leg after the slide-key call change, the interval
# farms (ext + reconnect) and the local-client GPU suites
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r05ac}
mkdir -p $O
timeout -k 10 300 python3 -u tools/local_leg.py 0 > $O/local.json 2> $O/local.err || exit 1
MTE_HTREE_LDS=0 timeout -k 10 300 python3 -u tools/lc_probe.py > $O/probe.json 2> $O/probe.err || exit 1
timeout -k 10 200 node tests/node/interval_farm.js ext > $O/farm_ext.json 2> $O/farm_ext.err || exit 1
timeout -k 10 300 node tests/node/interval_farm.js reconnect > $O/farm_rec.json 2> $O/farm_rec.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_local_refs.py tests/test_intervals.py tests/test_htree.py tests/test_reconnect.py tests/test_local_ops.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" > $O/rc.txt
