#!/bin/bash
# Build libmte.so variants from alternative source trees: build_var/<name>/src -> build_var/<name>/libmte.so
set -e
cd "$(dirname "$0")/.."
for d in build_var/*/src; do
  name=$(basename $(dirname $d))
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -I$d \
      -o build_var/$name/libmte.so $d/mte_engine.hip ) &
done
wait
ls -la build_var/*/libmte.so
