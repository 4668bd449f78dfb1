mkdir -p gpurun_out
for v in base vrec dpp both; do
  timeout -k 10 120 python tools/bench_var.py build_var/$v/libmte.so --docs 1250 --steps 10 --warmup 3 --no-tree-leg --no-node-leg --no-cpu-baseline > gpurun_out/v_${v}_1250.json 2>> gpurun_out/var.err || exit 1
  timeout -k 10 200 python tools/bench_var.py build_var/$v/libmte.so --steps 10 --warmup 3 --no-tree-leg --no-node-leg --no-cpu-baseline > gpurun_out/v_${v}_10k.json 2>> gpurun_out/var.err || exit 1
done
