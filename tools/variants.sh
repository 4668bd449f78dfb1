#!/bin/bash
# Build A/B variants of libmte.so into build_var/<name>/ (experiments only;
# the product library is fluidframework_amd/_lib/libmte.so).
set -e
cd "$(dirname "$0")/.."
build() {  # name flags...
  local name=$1; shift
  mkdir -p build_var/$name
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared "$@" \
    -o build_var/$name/libmte.so fluidframework_amd/csrc/mte_engine.hip &
}
rm -rf build_var
build e2w5 -DMTE_PASS1_EMAX=2 -DMTE_PAIR_WAVES=5
build e4w3 -DMTE_PASS1_EMAX=4 -DMTE_PAIR_WAVES=3
build e4w5 -DMTE_PASS1_EMAX=4 -DMTE_PAIR_WAVES=5
wait
ls -la build_var/*/libmte.so
