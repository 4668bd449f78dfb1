cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 900 python3 -u tools/varbench.py $VARIANTS > gpurun_out/var.log 2>&1 || { echo VARFAIL; tail gpurun_out/var.log; exit 1; }
cat gpurun_out/var.log
echo ALLOK
