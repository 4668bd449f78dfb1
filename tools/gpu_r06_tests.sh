#!/bin/bash
# round 6: the GPU suite (or the tests named in $TESTS) and smoke on the box;
# smoke only when the tests ran to an end (passed or failed, no fault / timeout)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r06t}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc" > $O/rc.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc" >> $O/rc.txt
exit $rc
