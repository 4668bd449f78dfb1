# Quick GPU iteration: parity tests, microbenchmarks, one bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python3 -u tools/microbench.py ${MICRO:-scale types} > gpurun_out/micro.log 2>&1 || { echo MICROFAIL; tail gpurun_out/micro.log; exit 1; }
cat gpurun_out/micro.log
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err || { echo BENCHFAIL; tail gpurun_out/bench_iter.err; exit 1; }
cat gpurun_out/bench_iter.json
echo ALLOK
