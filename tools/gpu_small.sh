cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for cfg in 2 4; do
timeout -k 10 300 python3 -u bench.py --config $cfg > gpurun_out/bench$cfg.json 2> gpurun_out/bench$cfg.err || { echo BENCHFAIL; tail -20 gpurun_out/bench$cfg.err; exit 1; }
python3 -c "import json;b=json.load(open('gpurun_out/bench$cfg.json'));print($cfg, b['value'],b['ms_per_step'],b['roofline']['frac'],b['parity_sample'])"
done
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/bench3.json 2> gpurun_out/bench3.err || { echo BENCHFAIL; tail -20 gpurun_out/bench3.err; exit 1; }
python3 -c "import json;b=json.load(open('gpurun_out/bench3.json'));print(3, b['value'],b['ms_per_step'])"
