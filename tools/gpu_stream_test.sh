cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "stream" > gpurun_out/gpu_stream.log 2>&1 || { echo STREAMFAIL; tail -30 gpurun_out/gpu_stream.log; exit 1; }
tail -8 gpurun_out/gpu_stream.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
echo ALLOK
