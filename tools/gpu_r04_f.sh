# round 4: relpos / interval host tests and the HBM tree pass's phase profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_relpos.py tests/test_intervals.py tests/test_node_host.py -m gpu -v \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc" > $O/rc.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/local_leg.py --prof 0 > $O/local_prof.json 2> $O/local_prof.err || exit 1
