cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in prio1 prio4; do
  MTE_WAVE_CLOCK=gpurun_out/wclock_$v.bin timeout -k 10 300 python3 -u tools/bench_var.py build_var/$v/libmte.so --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || { echo FAIL $v; tail -20 gpurun_out/bench_$v.err; exit 1; }
  echo "== $v"; python3 -c "import json;b=json.load(open('gpurun_out/bench_$v.json'));print(b['value'],b['ms_per_step'],b['roofline']['kernel_ms'],b['digest_fold'])"
  python3 tools/wave_clock.py gpurun_out/wclock_$v.bin
done
