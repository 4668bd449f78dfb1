#!/bin/bash
# round 5: interval farms (ext / reconnect, raw JSON), then the full GPU suite
# (no -x: every failure listed), smoke and the default bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r05f}
mkdir -p $O
timeout -k 10 200 node tests/node/interval_farm.js ext > $O/farm_ext.json 2> $O/farm_ext.err || exit 1
timeout -k 10 300 node tests/node/interval_farm.js reconnect > $O/farm_rec.json 2> $O/farm_rec.err || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests rc=$?" > $O/rc.txt
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || exit 1
P="python3 bench.py --no-cpu-baseline --no-tree-leg --no-local-leg"
timeout -k 10 300 $P > $O/bench3.json 2> $O/bench3.err || exit 1
echo done >> $O/rc.txt
