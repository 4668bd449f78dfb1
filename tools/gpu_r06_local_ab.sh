#!/bin/bash
# round 6: the HBM tree pass's register variants on the local-client leg
# (tools/local_leg.py), product build first, then build_var/<v> (MTE_LIB_DIR)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r06lab}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?
  echo "tests rc=$rc" >> $O/rc.txt
  [ $rc -le 1 ] || exit $rc
fi
for v in product $VARIANTS; do
  if [ "$v" = product ]; then D=""; else D="MTE_LIB_DIR=build_var/$v"; fi
  env $D timeout -k 10 300 python3 -u tools/local_leg.py 0 > $O/local_$v.json 2> $O/local_$v.err || exit 1
done
echo done >> $O/rc.txt
