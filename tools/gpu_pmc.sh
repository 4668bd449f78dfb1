# PMC instruction-mix probe of the replay kernels (one counter group per pass).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --ops ${OPS:-2000}"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace -d gpurun_out/pmc1 -o run --output-format csv -- $B > gpurun_out/pmc1.log 2>&1 || { echo PMC1FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVES SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_FLAT SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/pmc4 -o run --output-format csv -- $B > gpurun_out/pmc4.log 2>&1 || { echo PMC4FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc2 -o run --output-format csv -- $B > gpurun_out/pmc2.log 2>&1 || { echo PMC2FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc3 -o run --output-format csv -- $B > gpurun_out/pmc3.log 2>&1 || { echo PMC3FAIL; exit 1; }
echo ALLOK
