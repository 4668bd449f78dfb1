#!/bin/bash
# round 5: config 5 with the apply writing the column entries (cols skips carried documents)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r05ag}
mkdir -p $O
timeout -k 10 300 python3 -u bench.py --config 5 --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg > $O/bench5.json 2> $O/bench5.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_chunk.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" > $O/rc.txt
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/stats5 -o run --output-format csv -- python3 bench.py --config 5 --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg > $O/stats5.json 2> $O/stats5.err || exit 1
