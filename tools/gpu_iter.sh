cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/gpu_tests.log 2>&1 || { echo TESTFAIL; exit 1; }
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_iter.log 2>&1 || { echo BENCHFAIL; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_BUSY_CU_CYCLES --kernel-trace -d gpurun_out/pmc_iter -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_iter.log 2>&1 || { echo PMCFAIL; exit 1; }
echo ALLOK
