#!/bin/bash
# interval ext farm: full JSON of the first differences
set -o pipefail
mkdir -p gpurun_out/r04j
timeout -k 10 300 node tests/node/interval_farm.js ext > gpurun_out/r04j/ext.json 2> gpurun_out/r04j/ext.err
echo "rc=$?" > gpurun_out/r04j/rc.txt
