# Full GPU suite, then bench lines for configs 2 and 4, and a rocprof kernel
# summary of config 5.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python3 -u bench.py --config 2 > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { echo BENCH2FAIL; tail -20 gpurun_out/bench2.err; exit 1; }
cat gpurun_out/bench2.json
timeout -k 10 300 python3 -u bench.py --config 4 > gpurun_out/bench4.json 2> gpurun_out/bench4.err || { echo BENCH4FAIL; tail -20 gpurun_out/bench4.err; exit 1; }
cat gpurun_out/bench4.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python3 bench.py --config 5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof5.log 2>&1 || { echo PROF5FAIL; tail -20 gpurun_out/prof5.log; exit 1; }
echo ALLOK
