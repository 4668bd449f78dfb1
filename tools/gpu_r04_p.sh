#!/bin/bash
# the longest HBM-tree chains in LDS (a launch of their own): local line, probe, tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 300 python -u tools/lc_probe.py > $O/probe.json 2> $O/probe.err || exit 1
MTE_HTREE_LDS_LONG=0 timeout -k 10 300 python -u tools/lc_probe.py > $O/probe_off.json 2> $O/probe_off.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_htree.py tests/test_local_ops.py tests/test_reconnect.py tests/test_interval_rebase.py \
  tests/test_local_refs.py tests/test_relpos.py tests/test_intervals.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?" > $O/rc.txt
