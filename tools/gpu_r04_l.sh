#!/bin/bash
# round 4: interval reconnection (MTE_OP_REF b = 4 / 5), transient reads, the
# HBM tree pass suites
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_interval_rebase.py tests/test_local_refs.py tests/test_intervals.py \
  tests/test_htree.py tests/test_relpos.py tests/test_reconnect.py tests/test_local_ops.py \
  -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" > $O/rc.txt
