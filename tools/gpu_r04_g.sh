# round 4: grouped plane moves in the HBM tree pass (tests + phase profile), interval ext farms
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_intervals.py tests/test_htree.py tests/test_relpos.py tests/test_reconnect.py \
  -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc" > $O/rc.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/local_leg.py --prof 0 24576 > $O/local_prof.json 2> $O/local_prof.err || exit 1
