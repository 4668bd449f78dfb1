#!/bin/bash
# round 5: trace two interval farm clients (slide records vs the reference's events)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r05i}
mkdir -p $O
MTE_FARM_TRACE=1,1 timeout -k 10 200 node tests/node/interval_farm.js ext 2 > $O/t_ext.json 2> $O/t_ext.err || exit 1
MTE_FARM_TRACE=1,2 timeout -k 10 200 node tests/node/interval_farm.js reconnect 2 > $O/t_rec.json 2> $O/t_rec.err || exit 1
echo done > $O/rc.txt
