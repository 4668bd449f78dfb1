cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MTE_WAVE_CLOCK=gpurun_out/wclock.bin timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_wc.json 2> gpurun_out/bench_wc.err || { echo FAIL; tail -20 gpurun_out/bench_wc.err; exit 1; }
python3 tools/wave_clock.py gpurun_out/wclock.bin
