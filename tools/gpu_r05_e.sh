#!/bin/bash
# round 5: full GPU suite + smoke on the current library, then the default bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r05e}
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests rc=$?" > $O/rc.txt
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || exit 1
P="python3 bench.py --no-cpu-baseline --no-tree-leg --no-local-leg"
timeout -k 10 300 $P > $O/bench3.json 2> $O/bench3.err || exit 1
timeout -k 10 300 $P --no-node-leg --config 5 > $O/bench5.json 2> $O/bench5.err || exit 1
echo done >> $O/rc.txt
