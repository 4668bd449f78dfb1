# PMC latency probe of the replay kernels: instruction-level accumulators
# (SQ_INST_LEVEL_* / SQ_INSTS_* = mean latency in cycles) and L2 hit rate.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --ops ${OPS:-2000}"
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmcl1 -o run --output-format csv -- $B > gpurun_out/pmcl1.log 2>&1 || { echo PMCL1FAIL; tail gpurun_out/pmcl1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/pmcl2 -o run --output-format csv -- $B > gpurun_out/pmcl2.log 2>&1 || { echo PMCL2FAIL; tail gpurun_out/pmcl2.log; exit 1; }
echo ALLOK
