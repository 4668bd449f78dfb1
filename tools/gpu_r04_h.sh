# round 4: the HBM tree pass fully inlined (no scratch, 6-7 waves / SIMD): tests, local line, kHE variant
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_htree.py tests/test_relpos.py tests/test_reconnect.py tests/test_local_ops.py \
  tests/test_local_refs.py tests/test_intervals.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc" > $O/rc.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/local_leg.py 0 24576 65536 > $O/local.json 2> $O/local.err || exit 1
MTE_LIB_DIR=$GRAFT_REPO_ROOT/build_var/khe2 timeout -k 10 300 python -u tools/local_leg.py 0 24576 > $O/local_khe2.json 2> $O/local_khe2.err || exit 1
