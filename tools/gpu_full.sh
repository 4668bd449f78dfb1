# Full GPU pass: parity tests, default bench, rocprof kernel-trace stats, PMC HBM bytes.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/gpu_tests.log; exit 1; }
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCHFAIL; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo PROFFAIL; tail -20 gpurun_out/prof.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 || { echo PMCFAIL; tail -20 gpurun_out/pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1 || { echo PMCFAIL; tail -20 gpurun_out/pmc_write.log; exit 1; }
echo ALLOK
