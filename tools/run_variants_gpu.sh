#!/bin/bash
# A/B variants of libmte.so (tools/variants.sh builds them into build_var/<name>/):
# config 3 at 10k docs and at 1,250 docs (the per-GPU share at N = 8), each
# variant loaded through MTE_LIB_DIR (fluidframework_amd/_native.py).
# Usage: run_variants_gpu.sh name ...
mkdir -p gpurun_out
B="--steps 10 --warmup 3 --no-tree-leg --no-node-leg --no-local-leg --no-cpu-baseline"
for v in "$@"; do
  MTE_LIB_DIR=build_var/$v timeout -k 10 200 python bench.py $B > gpurun_out/v_${v}_10k.json 2>> gpurun_out/var.err || exit 1
  MTE_LIB_DIR=build_var/$v timeout -k 10 120 python bench.py $B --docs 1250 > gpurun_out/v_${v}_1250.json 2>> gpurun_out/var.err || exit 1
done
