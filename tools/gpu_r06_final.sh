#!/bin/bash
# round-6 final library: GPU suite, smoke, the full bench, kernel stats and PMC
# traffic of configs 3 and 5, configs 2 / 4, the 1,250-document point and the
# local-client leg (side legs off where a profile needs the timed launch last)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r06final}
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?
  echo "tests rc=$rc" > $O/rc.txt
  [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench_full.json 2> $O/bench_full.err || exit 1
P="python3 bench.py --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/stats3 -o run --output-format csv -- $P > $O/stats3.json 2> $O/stats3.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc3/fetch -o run --output-format csv -- $P --steps 1 --warmup 0 > $O/pmc3_fetch.json 2> $O/pmc3_fetch.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc3/write -o run --output-format csv -- $P --steps 1 --warmup 0 > $O/pmc3_write.json 2> $O/pmc3_write.err || exit 1
timeout -k 10 400 python3 -u bench.py --config 5 --no-tree-leg --no-node-leg --no-local-leg > $O/bench5.json 2> $O/bench5.err || exit 1
P5="$P --config 5"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/stats5 -o run --output-format csv -- $P5 > $O/stats5.json 2> $O/stats5.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc5/fetch -o run --output-format csv -- $P5 --steps 1 --warmup 0 > $O/pmc5_fetch.json 2> $O/pmc5_fetch.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc5/write -o run --output-format csv -- $P5 --steps 1 --warmup 0 > $O/pmc5_write.json 2> $O/pmc5_write.err || exit 1
timeout -k 10 300 $P --config 2 > $O/bench2.json 2> $O/bench2.err || exit 1
timeout -k 10 300 $P --config 4 > $O/bench4.json 2> $O/bench4.err || exit 1
timeout -k 10 300 $P --docs 1250 > $O/bench_1250.json 2> $O/bench_1250.err || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/stats_local -o run --output-format csv -- python3 tools/local_leg.py 0 > $O/local.json 2> $O/local.err || exit 1
echo done >> $O/rc.txt
