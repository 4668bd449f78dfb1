#!/bin/bash
# A/B variants of libmte.so (tools/variants.sh builds them into build_var/<name>/):
# config 3 at 10k docs and at 1,250 docs (the per-GPU share at N = 8), each variant.
# Usage: run_variants_gpu.sh name ...
mkdir -p gpurun_out
for v in "$@"; do
  timeout -k 10 200 python tools/bench_var.py build_var/$v/libmte.so --steps 10 --warmup 3 --no-tree-leg --no-node-leg --no-cpu-baseline > gpurun_out/v_${v}_10k.json 2>> gpurun_out/var.err || exit 1
  timeout -k 10 120 python tools/bench_var.py build_var/$v/libmte.so --docs 1250 --steps 10 --warmup 3 --no-tree-leg --no-node-leg --no-cpu-baseline > gpurun_out/v_${v}_1250.json 2>> gpurun_out/var.err || exit 1
done
