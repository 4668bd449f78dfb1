# round-3 final library (last build): GPU suite, smoke, full bench, kernel
# stats and PMC traffic of configs 3 and 5 (side legs off, so the timed launch
# is the last one)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03final3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench_full.json 2> $O/bench_full.err || exit 1
P="python3 bench.py --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/stats3 -o run --output-format csv -- $P > $O/stats3.json 2> $O/stats3.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc3/fetch -o run --output-format csv -- $P --steps 1 --warmup 0 > $O/pmc3_fetch.json 2> $O/pmc3_fetch.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc3/write -o run --output-format csv -- $P --steps 1 --warmup 0 > $O/pmc3_write.json 2> $O/pmc3_write.err || exit 1
P5="$P --config 5 --steps 1 --warmup 0"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc5/fetch -o run --output-format csv -- $P5 > $O/pmc5_fetch.json 2> $O/pmc5_fetch.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc5/write -o run --output-format csv -- $P5 > $O/pmc5_write.json 2> $O/pmc5_write.err || exit 1
