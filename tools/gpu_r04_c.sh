# round 4: the whole GPU suite with the HBM tree pass and the side-key packing, then the bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc" > $O/rc.txt
# test failures (rc 1) leave the GPU usable; a crash, abort or time limit does not
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-node-leg --no-tree-leg > $O/bench.json 2> $O/bench.err || exit 1
