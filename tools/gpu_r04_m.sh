#!/bin/bash
# interval reconnect farm: full JSON of the differences
set -o pipefail
mkdir -p gpurun_out/r04m
timeout -k 10 300 node tests/node/interval_farm.js reconnect > gpurun_out/r04m/rec.json 2> gpurun_out/r04m/rec.err
echo "rc=$?" > gpurun_out/r04m/rc.txt
