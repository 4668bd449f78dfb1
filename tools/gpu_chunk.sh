# Chunked-pass iteration: its GPU tests, then the rest of the GPU suite, then a
# config-3 regression bench and a reduced config-5 bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chunk.py -x -v --timeout 120 --timeout-method thread > gpurun_out/chunk_tests.log 2>&1 || { echo CHUNKFAIL; tail -40 gpurun_out/chunk_tests.log; exit 1; }
tail -3 gpurun_out/chunk_tests.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/bench3.json 2> gpurun_out/bench3.err || { echo BENCH3FAIL; tail -20 gpurun_out/bench3.err; exit 1; }
cat gpurun_out/bench3.json
timeout -k 10 300 python3 -u bench.py --config 5 --docs 16 --ops 65536 --steps 2 --warmup 1 --cpu-seconds 5 > gpurun_out/bench5s.json 2> gpurun_out/bench5s.err || { echo BENCH5FAIL; tail -20 gpurun_out/bench5s.err; exit 1; }
cat gpurun_out/bench5s.json
echo ALLOK
