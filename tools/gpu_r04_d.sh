# round 4: GPU suite (config 5 full size against the chunked restatement), the
# config-5 bench line (round-phase bytes, chunked cpu_baseline), the default bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc" > $O/rc.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --config 5 --no-node-leg --no-tree-leg > $O/bench5.json 2> $O/bench5.err || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
