#!/bin/bash
# round 6: bench lines of the product library under environment knobs
#   ENVS="MTE_TREE_ROUNDS=8 MTE_TREE_ROUNDS=32" BENCH_ARGS="..." OUT=name
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-r06env}
mkdir -p $O
for e in default $ENVS; do
  if [ "$e" = default ]; then D=""; else D="$e"; fi
  env $D timeout -k 10 300 python3 -u bench.py $BENCH_ARGS > $O/bench_$e.json 2> $O/bench_$e.err
  rc=$?
  echo "bench $e rc=$rc" >> $O/rc.txt
  [ $rc -eq 0 ] || exit 1
done
echo done >> $O/rc.txt
