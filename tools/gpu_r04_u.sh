#!/bin/bash
# the default bench line on the final tree (traffic read from profiles/r04/final)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04u
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
echo "bench rc=$?" > $O/rc.txt
