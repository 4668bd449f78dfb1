#!/bin/bash
# Build A/B variants of libmte.so into build_var/<name>/ (experiments only; the
# product library is fluidframework_amd/_lib/libmte.so).  The flat-pass
# and chunk-pass translation units are rebuilt with the variant's flags and
# linked with the product's other objects (make -C fluidframework_amd/csrc first).
# Usage: variants.sh name:"flags" ...   e.g. variants.sh w5e2:"-DMTE_PASS1_EMAX=2"
set -e
cd "$(dirname "$0")/.."
OBJ=fluidframework_amd/_lib/obj
rm -rf build_var
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p build_var/$name
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c \
      -o build_var/$name/flat.o fluidframework_amd/csrc/mte_pass_flat.hip &&
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c \
      -o build_var/$name/chunk.o fluidframework_amd/csrc/mte_pass_chunk.hip &&
    /opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o build_var/$name/libmte.so \
      $OBJ/mte_engine.o $OBJ/mte_pass_tree.o $OBJ/mte_pass_htree.o build_var/$name/flat.o build_var/$name/chunk.o $OBJ/mte_build.o \
      -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib ) &
done
wait
ls -la build_var/*/libmte.so
