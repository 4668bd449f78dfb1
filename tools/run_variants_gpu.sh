#!/bin/bash
# A/B variants of libmte.so (tools/variants.sh builds them into build_var/<name>/):
# 1,250 docs of config 3 (the per-GPU share at N = 8) and config 2, each variant.
# Usage: run_variants_gpu.sh name ...
mkdir -p gpurun_out
for v in "$@"; do
  timeout -k 10 120 python tools/bench_var.py build_var/$v/libmte.so --docs 1250 --steps 10 --warmup 3 --no-tree-leg --no-node-leg --no-cpu-baseline > gpurun_out/v_${v}_1250.json 2>> gpurun_out/var.err || exit 1
  timeout -k 10 120 python tools/bench_var.py build_var/$v/libmte.so --config 2 --steps 20 --warmup 3 --no-tree-leg --no-node-leg --no-cpu-baseline > gpurun_out/v_${v}_c2.json 2>> gpurun_out/var.err || exit 1
done
