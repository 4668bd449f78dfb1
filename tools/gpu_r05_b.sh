#!/bin/bash
# round 5: wave timeline at 1,250 documents, and the early-props variant A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05b
mkdir -p $O
P="python3 bench.py --no-cpu-baseline --no-tree-leg --no-node-leg --no-local-leg"
MTE_WAVE_CLOCK=$O/wclock_1250.bin timeout -k 10 120 $P --docs 1250 --steps 1 --warmup 1 > $O/wc.json 2> $O/wc.err || exit 1
python3 tools/wave_clock.py $O/wclock_1250.bin > $O/wclock_1250.txt || exit 1
for v in base ep; do
  if [ $v = base ]; then D=fluidframework_amd/_lib; else D=build_var/$v; fi
  MTE_LIB_DIR=$D timeout -k 10 200 $P --docs 1250 > $O/b1250_$v.json 2> $O/b1250_$v.err || exit 1
  MTE_LIB_DIR=$D timeout -k 10 200 $P > $O/b3_$v.json 2> $O/b3_$v.err || exit 1
done
echo done > $O/rc.txt
