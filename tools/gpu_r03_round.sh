# chunked-pass round phases: chunk GPU tests, config 5 bench and kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03round7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_chunk.py -x -v --timeout 300 --timeout-method thread > $O/chunk_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --config 5 --steps 3 --warmup 1 > $O/bench5_round.json 2> $O/bench5_round.err || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/stats5 -o run --output-format csv -- python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline --no-local-leg --no-tree-leg > $O/stats5.json 2> $O/stats5.err || exit 1
