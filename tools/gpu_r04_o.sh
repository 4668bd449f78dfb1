#!/bin/bash
# local-client line: doc-count probe with LDS residency (chain latency)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04o
mkdir -p $O
for L in 0 24576 65536; do
  MTE_HTREE_LDS=$L timeout -k 10 300 python -u tools/lc_probe.py > $O/probe_$L.json 2> $O/probe_$L.err || exit 1
done
echo done > $O/rc.txt
