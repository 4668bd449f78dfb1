# round-3 final library, part B: configs 5 (+ PMC traffic), 2, 4 and the
# 1,250-document point
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03final2
mkdir -p $O
timeout -k 10 400 python -u bench.py --config 5 --steps 3 --warmup 1 > $O/bench5.json 2> $O/bench5.err || exit 1
P5="python3 bench.py --config 5 --no-cpu-baseline --steps 1 --warmup 0"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/stats5 -o run --output-format csv -- $P5 > $O/stats5.json 2> $O/stats5.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc5/fetch -o run --output-format csv -- $P5 > $O/pmc5_fetch.json 2> $O/pmc5_fetch.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc5/write -o run --output-format csv -- $P5 > $O/pmc5_write.json 2> $O/pmc5_write.err || exit 1
timeout -k 10 300 python -u bench.py --config 2 > $O/bench2.json 2> $O/bench2.err || exit 1
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline > $O/bench4.json 2> $O/bench4.err || exit 1
timeout -k 10 300 python -u bench.py --docs 1250 --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg > $O/bench_1250.json 2> $O/bench_1250.err || exit 1
