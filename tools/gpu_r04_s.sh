#!/bin/bash
# the Node host's combining ops and its suites after the packer change
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_combining.py tests/test_node_host.py tests/test_intervals.py tests/test_local_refs.py \
  -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" > $O/rc.txt
