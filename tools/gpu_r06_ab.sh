#!/bin/bash
# round 6: named GPU tests, then A/B bench lines of variant libraries
# (build_var/<name>/libmte.so through MTE_LIB_DIR) against the product build.
#   TESTS="tests/x.py::t ..." VARIANTS="t3 ..." BENCH_ARGS="..." OUT=name
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r06ab}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  echo "tests rc=$?" >> $O/rc.txt
fi
for v in product $VARIANTS; do
  if [ "$v" = product ]; then D=""; else D="MTE_LIB_DIR=build_var/$v"; fi
  env $D timeout -k 10 300 python3 -u bench.py $BENCH_ARGS > $O/bench_$v.json 2> $O/bench_$v.err
  rc=$?
  echo "bench $v rc=$rc" >> $O/rc.txt
  [ $rc -eq 0 ] || exit 1
done
echo done >> $O/rc.txt
