# iteration: GPU suite, config-3 regression bench, reduced + full config-5 benches
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/bench3.json 2> gpurun_out/bench3.err || { echo BENCH3FAIL; tail -20 gpurun_out/bench3.err; exit 1; }
cat gpurun_out/bench3.json
timeout -k 10 300 python3 -u bench.py --config 5 --docs 16 --ops 65536 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench5s.json 2> gpurun_out/bench5s.err || { echo BENCH5FAIL; tail -20 gpurun_out/bench5s.err; exit 1; }
cat gpurun_out/bench5s.json
timeout -k 10 600 python3 -u bench.py --config 5 --steps 2 --warmup 1 > gpurun_out/bench5.json 2> gpurun_out/bench5.err || { echo BENCH5FULLFAIL; tail -20 gpurun_out/bench5.err; exit 1; }
cat gpurun_out/bench5.json
echo ALLOK
