# small-batch round phases, variant library build_var/rs2 (halving retries,
# zamboni folded into the write-back): tests, 1,250 docs / config 2 A/B, diag
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03rsmall8
mkdir -p $O
export MTE_LIB_DIR=$GRAFT_REPO_ROOT/build_var/rs2
timeout -k 10 600 python -u -m pytest tests/test_gpu_rsmall.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="--no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg"
MTE_RSMALL=1 timeout -k 10 300 python -u bench.py --docs 1250 $B > $O/bench_1250.json 2> $O/bench_1250.err || exit 1
MTE_RSMALL=1 timeout -k 10 300 python -u bench.py --config 2 $B > $O/bench2.json 2> $O/bench2.err || exit 1
MTE_RSMALL=1 timeout -k 10 300 python -u bench.py --docs 2500 $B > $O/bench_2500.json 2> $O/bench_2500.err || exit 1
MTE_RSMALL=1 MTE_WAVE_CLOCK=/tmp/wclock.bin timeout -k 10 300 python -u tools/rsmall_diag.py 1250 > $O/diag.json 2> $O/diag.err || exit 1
MTE_RSMALL=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 bench.py --docs 1250 $B > $O/stats.json 2> $O/stats.err || exit 1
