# round-3 final library, part A: GPU suite, smoke, local-client probe, full
# bench (config 3, every side leg), kernel stats and PMC traffic of config 3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03final2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/lc_probe.py > $O/lc_probe.jsonl 2> $O/lc_probe.err || exit 1
timeout -k 10 600 python -u bench.py > $O/bench_full.json 2> $O/bench_full.err || exit 1
P="python3 bench.py --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/stats3 -o run --output-format csv -- $P > $O/stats3.json 2> $O/stats3.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc3/fetch -o run --output-format csv -- $P --steps 1 --warmup 0 > $O/pmc3_fetch.json 2> $O/pmc3_fetch.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc3/write -o run --output-format csv -- $P --steps 1 --warmup 0 > $O/pmc3_write.json 2> $O/pmc3_write.err || exit 1
