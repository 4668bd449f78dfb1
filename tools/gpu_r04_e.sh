# round 4: relative positions, regen group release and LDS-resident HBM tree
# documents on the GPU: their tests, then the local-client line per LDS budget
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_relpos.py tests/test_htree.py tests/test_reconnect.py \
  tests/test_local_ops.py tests/test_local_refs.py tests/test_deltas.py -m gpu -v --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc" > $O/rc.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/local_leg.py 0 24576 40960 65536 > $O/local_leg.json 2> $O/local_leg.err || exit 1
