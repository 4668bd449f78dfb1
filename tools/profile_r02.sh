#!/bin/bash
# Round profile of the headline workload (config 3) on the current libmte.so:
# rocprofv3 kernel statistics of a bench run, then the two PMC passes
# (FETCH_SIZE, WRITE_SIZE; one counter block each) that tools/pmc_traffic.py
# turns into HBM bytes per launch.  Writes under gpurun_out/prof_r02/.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/prof_r02
mkdir -p $out
B="python3 bench.py --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- $B --steps 5 --warmup 1 > $out/stats_bench.json 2> $out/stats.err
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/fetch -o run --output-format csv -- $B --steps 1 --warmup 0 > $out/fetch_bench.json 2> $out/fetch.err
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/write -o run --output-format csv -- $B --steps 1 --warmup 0 > $out/write_bench.json 2> $out/write.err
find $out -name "*.csv" | head -20
# the local-client side line's stream_kernel, on its own (a tiny headline job beside it)
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $out/local -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-tree-leg --no-node-leg --docs 256 --ops 1000 --steps 2 --warmup 0 > $out/local_bench.json 2> $out/local.err
