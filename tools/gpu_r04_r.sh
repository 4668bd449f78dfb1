#!/bin/bash
# combining ops on the GPU, the tree-pass suites around them, the local-client probe
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_combining.py tests/test_htree.py tests/test_local_ops.py tests/test_relpos.py \
  tests/test_local_refs.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" > $O/rc.txt
timeout -k 10 300 python -u tools/lc_probe.py > $O/probe.json 2> $O/probe.err
echo "probe rc=$?" >> $O/rc.txt
