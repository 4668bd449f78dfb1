#!/bin/bash
# round 5: interval farms (slide order) + the reference / interval GPU tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r05h}
mkdir -p $O
timeout -k 10 200 node tests/node/interval_farm.js ext > $O/farm_ext.json 2> $O/farm_ext.err || exit 1
timeout -k 10 300 node tests/node/interval_farm.js reconnect > $O/farm_rec.json 2> $O/farm_rec.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_local_refs.py tests/test_intervals.py tests/test_gpu_chunk.py tests/test_nan_merge.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" > $O/rc.txt
