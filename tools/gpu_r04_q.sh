#!/bin/bash
# StayOnRemove reference farms on the GPU (Python and Node hosts)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_local_refs.py tests/test_htree.py tests/test_node_host.py -k "stay or local_references" \
  -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" > $O/rc.txt
