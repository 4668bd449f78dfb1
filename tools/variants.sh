#!/bin/bash
# Build A/B variants of libmte.so into build_var/<name>/ (experiments only;
# the product library is fluidframework_amd/_lib/libmte.so).
# Usage: variants.sh name:"flags" ...
set -e
cd "$(dirname "$0")/.."
rm -rf build_var
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p build_var/$name
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared $flags \
    -o build_var/$name/libmte.so fluidframework_amd/csrc/mte_engine.hip &
done
wait
ls -la build_var/*/libmte.so
